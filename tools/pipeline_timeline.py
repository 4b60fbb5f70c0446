#!/usr/bin/env python3
"""Timeline of the pipelined C2 steps from a rocprofv3 kernel trace: per stream, the kernels of
the last timed steps with start / end relative to the step window, and for each kernel type the
union of its busy intervals (how long at least one launch of it was running) vs the step time.
Usage: pipeline_timeline.py <kernel_trace.csv> [steps]"""
import csv
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1])) if not r["Kernel_Name"].startswith("__amd")]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
short = lambda n: n.split("(")[0].replace("void ", "").split("::")[-1].split("<")[0]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
fb = [r for r in rows if short(r["Kernel_Name"]) == "fast_blur_kernel"]
# the last nsteps * 3 fast_blur launches delimit the window (3 engines per step)
k = 3 * nsteps
t0 = int(fb[-k]["Start_Timestamp"]) - 1
t1 = max(int(r["End_Timestamp"]) for r in rows)
win = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
span = (t1 - t0) / 1e3
print(f"window {span:.1f} us for ~{nsteps} steps ({span / nsteps:.1f} us/step)")
busy = defaultdict(list)
for r in win:
    busy[short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
def union(iv):
    iv.sort(); tot = 0; cs, ce = iv[0]
    for s, e in iv[1:]:
        if s > ce: tot += ce - cs; cs, ce = s, e
        else: ce = max(ce, e)
    return tot + ce - cs
allv = [iv for v in busy.values() for iv in v]
print(f"any kernel running: {union(list(allv)) / 1e3 / span:.3f} of the window")
for name, iv in sorted(busy.items(), key=lambda kv: -union(list(kv[1]))):
    print(f"{name:24s} launches {len(iv):3d}  busy-union {union(list(iv)) / 1e3:8.1f} us ({union(list(iv)) / 1e3 / span:.2f})  sum {sum(e - s for s, e in iv) / 1e3:8.1f} us")
# concurrency of fast_blur with others
print("per-stream sequence of the last step:")
last = [r for r in win if int(r["Start_Timestamp"]) >= int(fb[-3]["Start_Timestamp"]) - 1]
for sid in sorted({r["Stream_Id"] for r in last}):
    seq = [r for r in last if r["Stream_Id"] == sid]
    print(f" stream {sid}: " + ", ".join(f"{short(r['Kernel_Name'])}[{(int(r['Start_Timestamp']) - t0) / 1e3:.0f}-{(int(r['End_Timestamp']) - t0) / 1e3:.0f}]" for r in seq))
