#!/usr/bin/env python3
"""Quadtree tie pin vs real glibc heap addresses (VERDICT r2 "next" item 4).

ORBextractor::DistributeOctTree breaks equal-size ties by ExtractorNode* address
(ORBextractor.cc:934-938); the oracle pins creation order (orb_oracle.c:524-539). The harness
oracle/tools/qt_glibc_order.cpp restates DistributeOctTree over a real std::list<ExtractorNode>
(the reference's node layout and allocation sequence), sorts by the real pointers, and runs every
image in a fresh std::thread, L and R of a stereo frame concurrently (Frame.cc:144-153), in three
allocation contexts (DistributeOctTree alone; + ComputeKeyPointsOctTree's vectors; + operator()'s
cv::Mat traffic). This script feeds it the oracle's per-level FAST candidates of the C2 stream and
reports, per context, how often the real-address result equals the creation-order pin: per level
(keypoint order and kept set), per image (kept set), and per equal-size pair of the final-phase
sorts (address order == creation order).

Oracle / CPU only (test infrastructure):
    python tools/qt_glibc_order.py [--frames 16] [--out profiles/r02_parity_exposure.json]
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
import oracle  # noqa: E402
from orbslam2_amd import synth  # noqa: E402

EDGE_THRESHOLD = 19
MAXL = 16


class QtgLevel(C.Structure):
    _fields_ = [("cand", C.c_void_p), ("ncand", C.c_int), ("cell_counts", C.c_void_p), ("ncells", C.c_int),
                ("minX", C.c_int), ("maxX", C.c_int), ("minY", C.c_int), ("maxY", C.c_int), ("N", C.c_int),
                ("lw", C.c_int), ("lh", C.c_int)]


class QtgImage(C.Structure):
    _fields_ = [("nlevels", C.c_int), ("nfeatures", C.c_int), ("lev", QtgLevel * MAXL),
                ("out", C.c_void_p * MAXL), ("out_cap", C.c_int), ("nout", C.c_int * MAXL)]


def harness():
    oracle.build()
    L = C.CDLL(str(ROOT / "oracle" / "_build" / "libqt_glibc.so"))
    L.qtg_run_frames.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    return L


def level_inputs(img, nfeat=2000):
    """Per level: (candidates, cell counts, bounds, N, (w, h)) as ComputeKeyPointsOctTree sees them."""
    ex = oracle.Extractor(nfeat)
    ex.extract(img)
    out = []
    for l in range(ex.nlevels):
        cand, counts = ex.level_candidates_cells(l)
        lw, lh = ex.s.lw[l], ex.s.lh[l]
        b = (EDGE_THRESHOLD - 3, lw - EDGE_THRESHOLD + 3, EDGE_THRESHOLD - 3, lh - EDGE_THRESHOLD + 3)
        out.append((cand, counts, b, ex.features_per_level[l], (lw, lh)))
    return out


def run(L, inputs, ctx, pin, nfeat=2000):
    """Run the harness over all images (two per frame); -> per image list of per-level outputs, stats."""
    n = len(inputs)
    imgs = (QtgImage * n)()
    keep = []
    outs = []
    for i, levels in enumerate(inputs):
        im = imgs[i]
        im.nlevels = len(levels)
        im.nfeatures = nfeat
        im.out_cap = 4096
        lo = []
        for l, (cand, counts, b, N, (lw, lh)) in enumerate(levels):
            o = np.zeros(4096, oracle.KP_DTYPE)
            lo.append(o)
            lv = im.lev[l]
            lv.cand, lv.ncand = cand.ctypes.data, len(cand)
            lv.cell_counts, lv.ncells = counts.ctypes.data, len(counts)
            lv.minX, lv.maxX, lv.minY, lv.maxY = b
            lv.N, lv.lw, lv.lh = N, lw, lh
            im.out[l] = o.ctypes.data
        outs.append(lo)
        keep.append(lo)
    st = np.zeros(4, np.int64)
    if L.qtg_run_frames(imgs, n, 2, ctx, pin, st.ctypes.data) != 0:
        raise RuntimeError("qtg_run_frames failed")
    res = [[outs[i][l][: imgs[i].nout[l]].copy() for l in range(imgs[i].nlevels)] for i in range(n)]
    return res, {"final_phase_sorts": int(st[0]), "equal_size_pairs": int(st[1]),
                 "pairs_address_order_eq_creation_order": int(st[2]), "levels_reaching_final_phase": int(st[3])}


def kset(levels):
    return {(float(k["x"]), float(k["y"]), l) for l, ks in enumerate(levels) for k in ks}


def compare(real, pin):
    lev_order = lev_set = lev = 0
    shared = []
    img_same = 0
    for ri, pi in zip(real, pin):
        same_img = True
        for rl, pl in zip(ri, pi):
            lev += 1
            o = rl.tobytes() == pl.tobytes()
            lev_order += o
            s = {(float(k["x"]), float(k["y"])) for k in rl} == {(float(k["x"]), float(k["y"])) for k in pl}
            lev_set += s
            same_img &= o
        img_same += same_img
        a, b = kset(ri), kset(pi)
        shared.append(len(a & b) / max(len(b), 1))
    return {"levels": lev, "levels_order_equal": lev_order, "levels_set_equal": lev_set,
            "images": len(real), "images_identical": img_same,
            "min_keypoint_set_shared": round(min(shared), 4), "mean_keypoint_set_shared": round(float(np.mean(shared)), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16, help="C2 stereo frames (t = 0.., seed 2 + t)")
    ap.add_argument("--out", help="parity exposure JSON to add the glibc_pointer_order entry to")
    args = ap.parse_args()
    L = harness()
    images = [im for t in range(args.frames) for im in synth.stereo_pair(376, 1241, t)]
    inputs = [level_inputs(im) for im in images]
    # the harness's pin run must reproduce the oracle's DistributeOctTree exactly
    pin_res, _ = run(L, inputs, 0, 1)
    for i, levels in enumerate(inputs):
        for l, (cand, counts, b, N, _) in enumerate(levels):
            ref = oracle.distribute_octtree(cand, b[0], b[1], b[2], b[3], N)
            if ref.tobytes() != pin_res[i][l].tobytes():
                raise SystemExit(f"harness pin run != orc_distribute_octtree (image {i}, level {l})")
    oracle.set_tie_mode(1)
    rev = [[oracle.distribute_octtree(c, b[0], b[1], b[2], b[3], N) for (c, _, b, N, _) in lv] for lv in inputs]
    oracle.set_tie_mode(0)
    rep = {"workload": f"C2 stream: {args.frames} synthetic KITTI stereo frames (seed 2 + t), {2 * args.frames} "
                       "images, 8 levels each, ORBextractor(2000, 1.2, 8, 20, 7)",
           "harness": "oracle/tools/qt_glibc_order.cpp: real std::list<ExtractorNode> (72-B element, 88-B list "
                      "node), reference allocation sequence, std::sort on pair<int, ExtractorNode*>, one fresh "
                      "std::thread per image, L and R concurrently; glibc of this container "
                      "(tcache + fastbins for the node's 96-B chunk class)",
           "pin_check": "harness with creation-order ties == orc_distribute_octtree on every level",
           "contexts": {}}
    names = {0: "DistributeOctTree alone", 1: "+ ComputeKeyPointsOctTree vectors",
             2: "+ operator() cv::Mat traffic (pyramid, descriptors, blur clones)"}
    by_ctx = {}
    for ctx in (0, 1, 2):
        for rep_i in range(2):   # a second pass over the stream runs on warmed (reused) arenas
            real, st = run(L, inputs, ctx, 0)
            by_ctx.setdefault(ctx, real)
            c = compare(real, pin_res)
            c.update(st)
            c["vs_reversed_creation_order"] = compare(real, rev)
            key = f"ctx{ctx}_pass{rep_i}"
            c["context"] = names[ctx]
            rep["contexts"][key] = c
            print(key, json.dumps(c), flush=True)
    # does the real order depend on the allocation history around DistributeOctTree?
    rep["ctx_vs_ctx"] = {f"ctx{a}_vs_ctx{b}": compare(by_ctx[a], by_ctx[b]) for a, b in ((0, 1), (0, 2), (1, 2))}
    print(json.dumps(rep["ctx_vs_ctx"]), flush=True)
    pairs = sum(v["equal_size_pairs"] for v in rep["contexts"].values())
    agree = sum(v["pairs_address_order_eq_creation_order"] for v in rep["contexts"].values())
    rep["equal_size_pairs_total"] = pairs
    rep["address_order_eq_creation_order_frac"] = round(agree / max(pairs, 1), 4)
    if args.out:
        p = Path(args.out)
        doc = json.loads(p.read_text()) if p.exists() else {}
        doc["glibc_pointer_order"] = rep
        p.write_text(json.dumps(doc, indent=1) + "\n")
    print(json.dumps({k: v for k, v in rep.items() if k != "contexts"}, indent=1))


if __name__ == "__main__":
    main()
