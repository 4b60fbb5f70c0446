"""Per-kernel (and per-launch-shape) average durations from a rocprofv3 kernel trace CSV."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0]
    key = f"{name} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} lds={r['LDS_Block_Size']}"
    agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / len(v) / 1e3:9.1f} us x{len(v):4d}  {k}")
