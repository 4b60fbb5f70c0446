#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into profiles/pmc_traffic.json.

HBM bytes per launch = (f * FETCH_SIZE + WRITE_SIZE) * 1024 with the read factor f of the kernel's
access pattern, calibrated on this MI355X (profiles/fetch_calib.json, tools/fetch_calib.sh):
MI355X_MICROARCH.md §HBM has FETCH_SIZE (KB) tally half the bytes of coalesced streaming reads
(f = 2, measured here for 4, 8 and 16 B per lane) and asks for a calibration of other patterns;
fast_blur_kernel's tile staging tallies every request at full size (f = 1). WRITE_SIZE is exact
for the stores measured. Other kernels keep f = 2 (uncalibrated); ratios between variants are exact.
Usage: pmc_summary.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <batch> <out.json> [<pmc_SQ_INSTS_VALU dir>]
With the optional SQ_INSTS_VALU pass, each kernel also gets its VALU wave-instructions per
launch (a wave64 VALU instruction occupies a 16-lane SIMD for 4 cycles).
With REQSIZE_DIR / REQSIZE_TAG in the environment (tools/pmc_reqsize.sh <tag> over the same
command, results under REQSIZE_DIR/rq_<tag>_*), each kernel also gets its exact L2 -> fabric bytes
from the request-size counters (32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B read, 64 WRREQ_64B +
32 (WRREQ - WRREQ_64B) written; tools/reqsize_summary.py): that figure becomes
hbm_bytes_per_launch, the measured read factor (exact read bytes / FETCH_SIZE bytes) replaces the
calibrated one, and the document carries step_traffic_bytes (every dispatch of a step).
The summary is stamped (tools/stamp.py) with the library's source hash, the commit (GIT_HEAD in
the environment), the batch per launch and the resize mode (RESIZE_MODE, default 0): bench.py
reports these counters only for the library and configuration they were measured on.
"""
import csv
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from stamp import stamp  # noqa: E402


def short(name: str) -> str:
    base = name.split("(")[0]
    return base.split("::")[-1]


def load(d: Path, counter: str):
    acc = defaultdict(list)
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


def main():
    fdir, wdir, batch, out = Path(sys.argv[1]), Path(sys.argv[2]), int(sys.argv[3]), Path(sys.argv[4])
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    valu = load(Path(sys.argv[5]), "SQ_INSTS_VALU") if len(sys.argv) > 5 else {}
    calib = Path(__file__).resolve().parent.parent / "profiles" / "fetch_calib.json"
    rf = json.loads(calib.read_text())["read_factor"] if calib.exists() else {"default": 2.0}
    res = {}
    rq = {}
    if os.environ.get("REQSIZE_DIR") and os.environ.get("REQSIZE_TAG"):
        from reqsize_summary import summarize
        rq = summarize(Path(os.environ["REQSIZE_DIR"]), os.environ["REQSIZE_TAG"])
    for k in sorted(set(fetch) | set(write)):
        fv, wv = fetch.get(k, []), write.get(k, [])
        f_avg = sum(fv) / len(fv) if fv else 0.0
        w_avg = sum(wv) / len(wv) if wv else 0.0
        res[k] = {"launches": max(len(fv), len(wv)), "FETCH_SIZE_KB": round(f_avg, 3),
                  "WRITE_SIZE_KB": round(w_avg, 3),
                  "read_factor": rf.get(k, rf["default"]),
                  "hbm_bytes_per_launch": int((rf.get(k, rf["default"]) * f_avg + w_avg) * 1024),
                  "hbm_bytes_per_launch_x2_rule": int((2 * f_avg + w_avg) * 1024)}
        if valu.get(k):
            res[k]["valu_insts_per_launch"] = int(sum(valu[k]) / len(valu[k]))
        q = rq.get(k)
        if q:
            res[k]["read_factor_calibrated"] = res[k]["read_factor"]
            res[k]["read_bytes_per_launch"] = q["read_bytes"]
            res[k]["write_bytes_per_launch"] = q["write_bytes"]
            res[k]["rdreq_per_launch"] = {s_: round(v_, 1) for s_, v_ in q["rdreq"].items()}
            if f_avg:
                res[k]["read_factor"] = round(q["read_bytes"] / (f_avg * 1024), 4)
            res[k]["hbm_bytes_per_launch"] = q["traffic_bytes"]
    st = stamp(batch=batch)
    if os.environ.get("STEPS_PROFILED"):   # bench steps (warmup included) the PMC run executed
        st["steps_profiled"] = int(os.environ["STEPS_PROFILED"])
    formula = ("(read_factor*FETCH_SIZE + WRITE_SIZE) * 1024 per launch (read_factor: profiles/fetch_calib.json; "
               "hbm_bytes_per_launch_x2_rule = the guide's streaming-read rule applied to every kernel)")
    if rq:
        formula = ("32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B + 64 WRREQ_64B + 32 (WRREQ - WRREQ_64B) per launch "
                   "(TCC_EA0 request counts, tools/pmc_reqsize.sh; read_factor = those read bytes / FETCH_SIZE bytes, "
                   "read_factor_calibrated = profiles/fetch_calib.json's factor for the pattern)")
    doc = {"stamp": st, "batch": batch, "formula": formula, "kernels": res}
    if rq and st.get("steps_profiled"):
        doc["step_traffic_bytes"] = int(sum(v["hbm_bytes_per_launch"] * v["launches"] for v in res.values())
                                        / st["steps_profiled"])
    out.write_text(json.dumps(doc, indent=1))
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
