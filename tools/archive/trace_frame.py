"""Timeline of one stereo frame from a rocprofv3 kernel trace of build/stereo_latency:
start offset (us, from the previous frame's last stereo kernel), duration, stream, kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 18
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "stereo_median_cut" in r["Kernel_Name"]]
a, b = idx[k], idx[k + 1]
base = int(rows[a]["End_Timestamp"])
for r in rows[a + 1:b + 1]:
    n = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
    print(f"{(int(r['Start_Timestamp']) - base) / 1e3:9.1f} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:7.1f}"
          f" s{r['Stream_Id']} {n} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}")
