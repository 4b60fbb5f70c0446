"""Overlap of the left / right ORBextractor kernel chains per stereo frame, from a rocprofv3
kernel trace of orb-slam2-noted_amd/build/stereo_latency (threads mode).

Each frame = the left engine's chain (resize x7, fast_blur, fast_nms, quadtree, describe) on its
stream, the right engine's chain on another stream, then the stereo kernels on the left stream.
A frame ends at its stereo_median_cut. Prints per-frame [L], [R] spans and their intersection,
and a JSON summary line (frames whose chains overlap, median overlap fraction of the shorter
chain, median frame GPU span)."""
import csv
import json
import sys
from statistics import median

rows = list(csv.DictReader(open(sys.argv[1])))
key = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
EXTRACT = ("resize_level_kernel", "fast_blur_kernel", "quadtree_kernel", "describe2_kernel", "describe_kernel")
frames, cur = [], []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].split("<")[0].split(" ")[-1].split("::")[-1]
    cur.append((name, r[key], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if name == "stereo_median_cut":
        frames.append(cur)
        cur = []
out = []
for f in frames:
    stereo_q = [q for n, q, a, b in f if n.startswith("stereo_")][0]
    ext = [(q, a, b) for n, q, a, b in f if n in EXTRACT]
    qs = sorted({q for q, _, _ in ext})
    if len(qs) != 2:
        out.append(None)
        continue
    span = {q: (min(a for qq, a, _ in ext if qq == q), max(b for qq, _, b in ext if qq == q)) for q in qs}
    L = span[stereo_q] if stereo_q in span else span[qs[0]]
    R = span[[q for q in qs if span[q] != L][0]]
    inter = max(0, min(L[1], R[1]) - max(L[0], R[0]))
    shorter = min(L[1] - L[0], R[1] - R[0])
    t0 = min(a for _, _, a, _ in f)
    t1 = max(b for _, _, _, b in f)
    out.append({"L_us": (L[1] - L[0]) / 1e3, "R_us": (R[1] - R[0]) / 1e3, "overlap_us": inter / 1e3,
                "overlap_frac": inter / shorter if shorter else 0.0, "gpu_span_us": (t1 - t0) / 1e3})
good = [o for o in out if o]
for i, o in enumerate(out):
    if o:
        print(f"frame {i:3d}: L {o['L_us']:7.1f} us  R {o['R_us']:7.1f} us  overlap {o['overlap_us']:7.1f} us "
              f"({100 * o['overlap_frac']:5.1f} % of the shorter)  frame GPU span {o['gpu_span_us']:7.1f} us")
print(json.dumps({"frames": len(out), "frames_two_streams": len(good),
                  "frames_overlapping": sum(1 for o in good if o["overlap_us"] > 0),
                  "median_overlap_frac": round(median(o["overlap_frac"] for o in good), 3) if good else None,
                  "median_gpu_span_us": round(median(o["gpu_span_us"] for o in good), 1) if good else None,
                  "stream_key": key}))
