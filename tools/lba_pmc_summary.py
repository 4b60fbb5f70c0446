"""Summarise a LocalBA MFMA PMC pass (rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 ...) against the per-kernel durations of a
separate --kernel-trace --stats run (PMC passes serialise and stretch kernels):
per kernel FP64 MFMA instructions and flops per launch, MFMA-busy SIMD cycles per launch, and
MFMA utilisation = busy / (duration x 2.4 GHz x SIMDs): chip-wide (1024 SIMDs) and, for
single-workgroup kernels, on the one CU that runs them (4 SIMDs).
    python tools/lba_pmc_summary.py <counter_collection.csv> <kernel_stats.csv> [out.json]"""
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from stamp import stamp  # noqa: E402
from collections import defaultdict

CLK, SIMDS = 2.4e9, 1024
cnt = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
grid = {}
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
    grid[k] = (int(r["Grid_Size"]), int(r["Workgroup_Size"]))
dur = {}
for r in csv.DictReader(open(sys.argv[2])):
    dur[r["Name"].split("(")[0].split("::")[-1]] = float(r["AverageNs"]) * 1e-9
out = {}
for k, v in cnt.items():
    n = len(disp[k])
    mf = v.get("SQ_INSTS_VALU_MFMA_F64", 0) / n
    if mf == 0 or k not in dur:
        continue
    busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / n
    d = dur[k]
    wgs = grid[k][0] // grid[k][1]
    e = {"launches_sampled": n, "avg_launch_us": round(d * 1e6, 3), "mfma_f64_insts_per_launch": round(mf, 1),
         "mfma_f64_flops_per_launch": round(v.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0) / n * 512),
         "mfma_busy_simd_cycles_per_launch": round(busy),
         "mfma_util_chip": round(busy / (d * CLK * SIMDS), 5),
         "mfma_tflops_while_running": round(v.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0) / n * 512 / d / 1e12, 3)}
    if wgs == 1:
        e["mfma_util_own_cu"] = round(busy / (d * CLK * 4), 4)
    out[k] = e
rep = {"stamp": stamp(), "source": sys.argv[1:3], "clock_hz": CLK, "kernels": out}
txt = json.dumps(rep, indent=1)
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(txt + "\n")
print(txt)
