#!/usr/bin/env python3
"""Benchmark: ORB extract + stereo match throughput (BASELINE.json metric) on MI355X.

Workload (BASELINE.json configs[1]): KITTI-like synthetic stereo pairs
1241x376, ORBextractor(2000, 1.2, 8, 20, 7) on left and right + Frame::ComputeStereoMatches
(KITTI00-02.yaml bf=386.1448, fx=718.856). One step = one batch of B stereo frames already
resident in HBM: 2B images through pyramid / FAST / blur / quadtree / IC_Angle+BRIEF, then
B stereo matches. The batch is split over `--engines` extraction engines on their own HIP
streams (orbx_pipeline_*), whose pyramid / FAST / blur phases run in turn so that one chunk's
VALU-bound phase overlaps the others' latency-bound ones. `value` = stereo frames/s over all ranks.

Multi-GPU (C5): one process per GPU (torchrun), each rank runs its own stream of batches
(weak scaling); the shared read-only extractor/camera state is broadcast from rank 0 once
over RCCL (torch.distributed nccl backend) before timing. No per-frame collective.

Also reported: `roofline` for the dominant kernel (hipEvent durations on each engine's
stream over the timed region; a launch processes B / engines pairs and shares the GPU with
the other engines' kernels) and `cpu_baseline` = the CPU oracle (single-threaded C
restatement, oracle/) on a bounded sample of the same workload, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues per process (HIP's default 4). The
# host-batch leg runs 2 engine streams + an H2D and a D2H copy stream next to torch's stream;
# with 4 queues copy streams share a queue with an engine, and the copies wait behind its
# kernels (value_e2e 48.9k -> 58.1k stereo frames/s with 8 queues). Must be set
# before the HIP runtime initialises; raised to at least 8 (a larger setting is kept).
try:
    _hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
except ValueError:
    _hwq = 4
os.environ["GPU_MAX_HW_QUEUES"] = str(max(_hwq, 8))

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))

KITTI_BF = 386.1448
KITTI_FX = 718.856
W, H = 1241, 376
NFEAT = 2000
BYTES_PER_STEREO_FRAME = 2 * W * H + 2 * NFEAT * (28 + 32) + NFEAT * 8   # 1,189,232 B
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
C3_BYTES_PER_FRAME = 640 * 480 + 1000 * 60 + 1000 * (4 + 8)   # 379,200 B per RGB-D frame


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_pool(n_pairs: int, rank: int, world: int):
    """C2 (one GPU): frames t = 0.. of the seed-2 stream (left seed 2 + t). C5 (world > 1):
    SURVEY §8d's eight independent streams, seeds 10..17, one per rank: rank r's frame t is
    generated from seed 10 + r + 8 t, so no two ranks share a frame."""
    from orbslam2_amd import synth
    POOL_SEEDS.clear()
    if world == 1:
        POOL_SEEDS.extend(2 + t for t in range(n_pairs))
        return [synth.stereo_pair(H, W, t) for t in range(n_pairs)]
    POOL_SEEDS.extend(10 + rank + 8 * t for t in range(n_pairs))
    return [synth.stereo_pair(H, W, 8 * t, base_seed=10 + rank) for t in range(n_pairs)]


POOL_SEEDS = []   # left-image generator seed of each pool pair (make_pool)


def host_cpu():
    """(usable host threads, CPU model) of this box; the GPU box's CPU share is 16 threads."""
    n = len(os.sched_getaffinity(0))
    n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return max(1, n), model


def cpu_baseline(pool, n_frames: int):
    """Time the CPU oracle (test infrastructure) on the C2 workload in SURVEY §8d's two modes:
    throughput (a thread pool over the host's cores, independent frames; the reported value) and
    single thread (one frame after another). The oracle's C calls release the GIL."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    oracle.build()
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))

    def run(k0, count):
        exL, exR = oracle.Extractor(NFEAT), oracle.Extractor(NFEAT)
        for i in range(k0, k0 + count):
            L, R = pool[i % len(pool)]
            kL, dL = exL.extract(L)
            kR, dR = exR.extract(R)
            oracle.stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, mb)

    t0 = time.perf_counter()
    run(0, n_frames)
    dt1 = time.perf_counter() - t0
    threads, model = host_cpu()
    per = max(2, n_frames // 2)
    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda k: run(k * per, per), range(threads)))
        dtn = time.perf_counter() - t0
    return {"value": round(threads * per / dtn, 3), "unit": "stereo frames/s", "cores": threads, "kind": "port",
            "sample": f"{threads * per} synthetic 1241x376 stereo frames (C2 generator, {len(pool)} distinct), "
                      f"oracle extract L+R + ComputeStereoMatches, {threads} threads x {per} frames, {dtn:.1f} s; "
                      f"host CPU {model}",
            "single_thread": {"value": round(n_frames / dt1, 3), "cores": 1,
                              "sample": f"{n_frames} frames one after another, {dt1:.1f} s"}}


def cpu_latency(pool, warmup: int, frames: int):
    """The oracle in SURVEY §8d's latency mode: per stereo frame the left and right extraction on
    two threads (Frame.cc:144-153 starts two std::threads per frame), then ComputeStereoMatches;
    median / mean wall time per frame. The oracle's C calls release the GIL."""
    import threading
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    oracle.build()
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    exL, exR = oracle.Extractor(NFEAT), oracle.Extractor(NFEAT)
    ms = []
    for t in range(warmup + frames):
        L, R = pool[t % len(pool)]
        res = {}
        t0 = time.perf_counter()
        tl = threading.Thread(target=lambda: res.__setitem__("L", exL.extract(L)))
        tr = threading.Thread(target=lambda: res.__setitem__("R", exR.extract(R)))
        tl.start(); tr.start(); tl.join(); tr.join()
        (kL, dL), (kR, dR) = res["L"], res["R"]
        oracle.stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, mb)
        if t >= warmup:
            ms.append(1000 * (time.perf_counter() - t0))
    a = np.array(ms)
    return {"median_ms": round(float(np.median(a)), 3), "mean_ms": round(float(a.mean()), 3),
            "frames": frames, "warmup": warmup, "cores": 2, "kind": "port",
            "sample": f"{frames} synthetic 1241x376 stereo frames ({len(pool)} distinct), oracle, L and R on two "
                      f"threads per frame + ComputeStereoMatches, {a.sum() / 1000:.1f} s"}


def bench_latency(amd, args, pool, with_cpu):
    """Drop-in latency (SURVEY §8d latency mode): the C++ host layer's
    ORBextractor L and R on two std::threads per frame + ComputeStereoMatches, host image in and
    host keypoints / descriptors / mvuRight / mvDepth out (tools/stereo_latency.cpp), 16 warm-up
    and 512 timed frames; `serial` runs L then R on one thread for comparison."""
    import subprocess
    import tempfile
    exe = ROOT / "orb-slam2-noted_amd" / "build" / "stereo_latency"
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    with tempfile.NamedTemporaryFile(suffix=".u8", delete=False) as f:
        for L, R in pool:
            f.write(np.ascontiguousarray(L).tobytes())
            f.write(np.ascontiguousarray(R).tobytes())
        path = f.name
    out = {}
    try:
        for mode, frames in (("threads", args.latency_frames), ("serial", max(64, args.latency_frames // 4))):
            r = subprocess.run([str(exe), path, str(len(pool)), str(W), str(H), str(NFEAT), repr(KITTI_BF), repr(mb),
                                str(args.latency_warmup), str(frames), mode], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError(f"stereo_latency {mode} failed: {r.stderr.strip()}")
            out[mode] = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        os.unlink(path)
    t = out["threads"]
    res = {"latency": {"workload": "C2 single stereo frame through the drop-in boundary: host 1241x376 L/R in, "
                                   "ORBextractor(2000) L || R on two std::threads (Frame.cc:144-153) + "
                                   "ComputeStereoMatches, host outputs",
                       "median_ms": t["median_ms"], "mean_ms": t["mean_ms"], "p90_ms": t["p90_ms"],
                       "frames": t["frames"], "warmup": t["warmup"],
                       "frames_per_s": round(1000.0 / t["mean_ms"], 2),
                       "serial_median_ms": out["serial"]["median_ms"], "serial_mean_ms": out["serial"]["mean_ms"]}}
    if with_cpu:
        res["latency"]["cpu_baseline"] = cpu_latency(pool, args.latency_warmup, args.cpu_latency_frames)
    return res


def bench_e2e(amd, args, pool, bf, mb):
    """C2 with host I/O: the same 384-pair batches from page-locked host
    memory through orbx_pipeline_stereo_batch_host -- H2D of batch k+1 on a copy stream overlapped
    with batch k's kernels, every engine's keypoints / descriptors / mvuRight / mvDepth copied back
    to page-locked host memory -- timed to the last output byte in host memory."""
    B = args.batch
    ins, outs = [], []
    for k in range(2):
        a = amd.host_empty((2 * B, H, W), np.uint8)
        for i in range(B):
            L, R = pool[(i + 3 * k) % len(pool)]
            if k:
                L, R = np.roll(L, 7 * k, axis=1), np.roll(R, 7 * k, axis=1)
            a[2 * i], a[2 * i + 1] = L, R
        ins.append(a)
    pl = amd.StereoPipeline(NFEAT, n_engines=args.e2e_engines)
    pl.reserve(W, H, B)
    cap = pl.capacity()
    outs = [amd.StereoHostBatch(B, cap) for _ in range(2)]

    def step(k):
        pl.stereo_batch_host(ins[k % 2], B, W, H, W, W * H, float(bf), mb, outs[k % 2])

    for k in range(args.warmup):
        step(k)
    pl.wait()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    pl.wait()
    dt = time.perf_counter() - t0
    kL = outs[(args.steps - 1) % 2].pair(0)
    if len(kL[0]) < 100 or int((kL[4] >= 0).sum()) < 10:
        raise RuntimeError("implausible host-mode output")
    h2d = 2 * B * W * H
    d2h = 2 * B * cap * (28 + 32 + 4) + 2 * B * cap * 4
    pl.close()
    return {"value_e2e": round(B * args.steps / dt, 2),
            "e2e": {"ms_per_step": round(1000 * dt / args.steps, 4), "stereo_frames_per_step": B,
                    "pipeline_engines": args.e2e_engines, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                    "h2d_bytes_per_step": h2d, "d2h_bytes_per_step": d2h,
                    "pcie_gbs": round((h2d + d2h) * args.steps / dt / 1e9, 2),
                    "note": "page-locked host images in, host keypoints / descriptors / mvuRight / mvDepth out; "
                            "PCIe-inclusive rate (value is the HBM-resident rate)"}}


def c2_buffers(B: int, nbufs: int, pool):
    """`nbufs` rotating resident batches of B stereo pairs (batch k: the pool rolled by 7k px, so
    no two batches are identical)."""
    import torch
    bufs = []
    for k in range(nbufs):
        imgs = np.empty((2 * B, H, W), np.uint8)
        for i in range(B):
            L, R = pool[(i + 3 * k) % len(pool)]
            if k:
                L = np.roll(L, 7 * k, axis=1)
                R = np.roll(R, 7 * k, axis=1)
            imgs[2 * i], imgs[2 * i + 1] = L, R
        bufs.append(torch.from_numpy(imgs).cuda())
    torch.cuda.synchronize()
    return bufs


def time_c2(amd, args, dist, params, bufs, resize_mode, steps, profile=False, blur_mode=None):
    """Warmup + `steps` timed batches of the C2 leg on a fresh pipeline; the timed region is
    bracketed by a barrier + device synchronisation on both sides. -> (elapsed s, profile, pipeline)."""
    import torch
    nf, sf, nl, ith, mth, bf, mb = params
    B = args.batch
    ex = amd.StereoPipeline(int(nf), float(sf), int(nl), int(ith), int(mth), n_engines=args.engines,
                            resize_mode=resize_mode, blur_mode=args.blur_mode if blur_mode is None else blur_mode)
    ex.reserve(W, H, B)

    def step(k):
        t = bufs[k % len(bufs)]
        ex.stereo_batch(t.data_ptr(), B, W, H, W, W * H, float(bf), mb)

    for k in range(args.warmup):
        step(k)
    amd.device_sync()
    if profile:
        ex.profile(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    amd.device_sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    amd.device_sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ex.profile_read() if profile else {}
    ex.profile(False)
    return elapsed, prof, ex


def bench_c2(amd, args, dist, world, params, pool):
    """C2 headline leg: B resident stereo pairs per step through the 3-engine pipeline, under
    `--resize-mode` (SURVEY A.2 pin (a) by default); the same leg under the other resize variant is
    reported beside it (`alt_resize_mode`)."""
    from orbslam2_amd import dist as odist
    B = args.batch
    bufs = c2_buffers(B, args.bufs, pool)
    elapsed, prof, ex = time_c2(amd, args, dist, params, bufs, args.resize_mode, args.steps,
                                profile=not args.no_profile)
    elapsed = odist.max_over_ranks(elapsed, COLL_DEV, dist)
    per_launch = B / len(ex.engines)   # stereo pairs one extraction / stereo launch processes

    # sanity: the batch produced keypoints and stereo matches
    k0 = ex.fetch(0)[0]
    u0, _ = ex.stereo_fetch(0)
    n_match = int((u0[: len(k0)] >= 0).sum())
    if len(k0) < 100 or n_match < 10:
        raise RuntimeError(f"implausible output: {len(k0)} keypoints, {n_match} stereo matches")
    engines = len(ex.engines)
    parity = c2_parity(ex, args, params, pool) if args.check_parity else None
    ex.close()

    frames = B * args.steps * world
    value = frames / elapsed
    ms_step = 1000 * elapsed / args.steps
    out = {
        "metric": "frames/sec ORB extract+match @1241x376 (1 GPU) + LocalBA keyframes/sec",
        "value": round(value, 2),
        "unit": "stereo frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": "C2: KITTI-like synthetic stereo 1241x376, ORBextractor(2000,1.2,8,20,7) L+R "
                        "+ Frame::ComputeStereoMatches",
            "stereo_frames_per_step_per_gpu": B,
            "pipeline_engines": engines,
            "image": f"{W}x{H}",
            "nfeatures": NFEAT,
            "resize_mode": args.resize_mode,
            "blur_mode": args.blur_mode,
            "blur_mode_meaning": "0 = OpenCV >= 3.4 fixed-point GaussianBlur rounding (SURVEY A.3 pin); 1 = OpenCV 3.2 "
                                 "SSE2 half-even column pass",
            "resize_mode_meaning": "0 = scalar FixedPtCast vertical pass (SURVEY A.2 (a), the oracle's default pin); "
                                   "1 = OpenCV 3.2 x86 SSE2 VResizeLinearVec_32s8u prefix (A.2 (b))",
            "streams": "seed-2 C2 stream" if world == 1 else "C5: rank r = seed 10 + r stream (seeds 10..17)",
            "parallelism": f"independent sequence per GPU x{world}",
            "keypoints_img0": int(len(k0)),
            "stereo_matches_img0": n_match,
        },
    }
    if prof:
        # the dominant kernel among those whose one launch processes a chunk's `per_launch` pairs (one
        # launch per chunk): the 7 per-level resize launches of a chunk each process one level, and
        # their summed duration is mostly the wait for the wave slots another engine's
        # fast_blur_kernel holds, so they are reported beside it, not as the unit kernel
        chunks = args.steps * engines
        unit = {k: v for k, v in prof.items() if v[1] == chunks}
        name, (tot, n) = max((unit or prof).items(), key=lambda kv: kv[1][0])
        avg_s = tot / n / 1000.0
        achieved = BYTES_PER_STEREO_FRAME * per_launch / avg_s / 1e9
        # counters from the committed PMC pass, only if it was measured on this library, batch and mode
        pmc, pmc_note = load_pmc_doc("pmc_traffic.json", amd.build_id(), batch=round(per_launch),
                                     resize_mode=args.resize_mode, blur_mode=args.blur_mode)
        ent = (pmc or {}).get(name, {})
        out["roofline"] = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 3),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                           "traffic": ent.get("hbm_bytes_per_launch"), "avg_launch_ms": round(tot / n, 4),
                           "algorithmic_bytes_per_launch": round(BYTES_PER_STEREO_FRAME * per_launch),
                           "pairs_per_launch": per_launch, "pmc_source": pmc_note}
        if ent.get("read_bytes_per_launch") is not None:
            out["roofline"]["traffic_formula"] = (
                "exact L2->fabric bytes per launch from the request-size counters: 32 RDREQ_32B + 64 RDREQ_64B + "
                "128 RDREQ_128B + 64 WRREQ_64B + 32 (WRREQ - WRREQ_64B) (tools/pmc_reqsize.sh)")
            out["roofline"]["traffic_read"] = ent["read_bytes_per_launch"]
            out["roofline"]["traffic_write"] = ent["write_bytes_per_launch"]
            out["roofline"]["read_factor_measured"] = ent.get("read_factor")
            out["roofline"]["traffic_x2_rule"] = ent.get("hbm_bytes_per_launch_x2_rule")
        elif ent.get("hbm_bytes_per_launch") is not None:
            out["roofline"]["traffic_formula"] = (f"(FETCH_SIZE x {ent.get('read_factor', 2.0)} + WRITE_SIZE) per launch, read factor "
                                                  "calibrated for this kernel's access pattern (profiles/fetch_calib.json)")
            out["roofline"]["traffic_x2_rule"] = ent.get("hbm_bytes_per_launch_x2_rule")
        step_tr = (pmc or {}).get("__step_traffic__")
        if step_tr:
            # every dispatch of a step (request-size counters), against SURVEY §8d's algorithmic bytes
            alg_step = BYTES_PER_STEREO_FRAME * B
            out["roofline"]["step_traffic_bytes"] = step_tr
            out["roofline"]["step_algorithmic_bytes"] = alg_step
            out["roofline"]["step_traffic_ratio"] = round(step_tr / alg_step, 3)
            out["roofline"]["step_traffic_gbs"] = round(step_tr / (ms_step / 1e3) / 1e9, 1)
        valu = ent.get("valu_insts_per_launch")
        if valu:   # the ceiling this integer kernel actually sits against
            out["roofline"]["valu_issue_frac"] = round(
                valu * VALU_CYCLES_PER_INST / (VALU_SIMDS * VALU_CLOCK_HZ) / (tot / n / 1e3), 4)
            out["roofline"]["valu_insts_per_launch"] = valu
        steps_prof = (pmc or {}).get("__stamp__", {}).get("steps_profiled")
        if pmc and steps_prof:
            # the whole step against VALU issue: every kernel dispatch of a step in the PMC pass (its
            # VALU instructions per dispatch x dispatches per step; the rocclr setup copies excluded)
            # x 4 cycles / (1024 SIMDs x 2.4 GHz), over this run's ms_per_step
            insts = sum(v["valu_insts_per_launch"] * v["launches"] / steps_prof for k, v in pmc.items()
                        if k != "__stamp__" and isinstance(v, dict) and not k.startswith("__amd_rocclr_copy") and "valu_insts_per_launch" in v)
            out["roofline"]["step_valu_insts"] = int(insts)
            out["roofline"]["step_valu_issue_frac"] = round(
                insts * VALU_CYCLES_PER_INST / (VALU_SIMDS * VALU_CLOCK_HZ) / (ms_step / 1e3), 4)
        # summed over the engines' launches, which overlap in time (so the sum exceeds ms_per_step)
        out["kernel_ms_per_step"] = {k: round(v[0] / args.steps, 4) for k, v in sorted(prof.items())}
        out["kernel_launches_per_step"] = {k: round(v[1] / args.steps, 3) for k, v in sorted(prof.items())}
        # the same launch (per_launch pairs) on one engine with nothing beside it: under the
        # pipeline a launch shares the CUs with the other engines' kernels, so its duration (and
        # `frac` above) measures the overlap as much as the kernel
        iso_ms = None if args.no_isolated else isolated_launch_ms(amd, params, bufs[0], round(per_launch), name,
                                                                   args.resize_mode)
        if iso_ms:
            iso = BYTES_PER_STEREO_FRAME * per_launch / (iso_ms / 1e3) / 1e9
            out["roofline"]["isolated"] = {"avg_launch_ms": round(iso_ms, 4), "achieved": round(iso, 3),
                                           "frac": round(iso / HBM_PEAK_GBS, 6),
                                           "note": "the same launch on one engine with nothing beside it; the "
                                                   "pipelined launch above shares the CUs with the next chunk's "
                                                   "resize and the previous chunk's quadtree / describe / stereo "
                                                   "for its whole duration (DESIGN.md §5, §5a)"}
            if valu:
                out["roofline"]["isolated"]["valu_issue_frac"] = round(
                    valu * VALU_CYCLES_PER_INST / (VALU_SIMDS * VALU_CLOCK_HZ) / (iso_ms / 1e3), 4)
    if parity is not None:
        out["parity_check"] = {"c2": gather_ranks(parity, dist)}
    if not args.no_alt_resize:
        alt = 1 - args.resize_mode
        a_el, _, a_ex = time_c2(amd, args, dist, params, bufs, alt, args.steps)
        a_ex.close()
        a_el = odist.max_over_ranks(a_el, COLL_DEV, dist)
        out["alt_resize_mode"] = {"resize_mode": alt, "value": round(frames / a_el, 2),
                                  "ms_per_step": round(1000 * a_el / args.steps, 4),
                                  "note": "the same leg (batches, steps, engines) under the other SURVEY A.2 "
                                          "vertical-pass variant; both variants are parity-tested on the GPU"}
        # the reference's documented platform (OpenCV 3.2.0 on x86-64, README.md:9): both SSE2 variants
        c_el, _, c_ex = time_c2(amd, args, dist, params, bufs, 1, args.steps, blur_mode=1)
        c_ex.close()
        c_el = odist.max_over_ranks(c_el, COLL_DEV, dist)
        out["alt_opencv32"] = {"resize_mode": 1, "blur_mode": 1, "value": round(frames / c_el, 2),
                               "ms_per_step": round(1000 * c_el / args.steps, 4),
                               "note": "the same leg under OpenCV 3.2's x86 SSE2 resize and GaussianBlur column "
                                       "passes (SURVEY A.2 (b) + A.3), the reference's documented platform"}
    del bufs   # the resident batches are not needed by the legs below
    return out


def gather_ranks(obj, dist):
    """Every rank's `obj`, in rank order (one all_gather_object; outside the timed regions)."""
    if dist is None:
        return [obj]
    lst = [None] * dist.get_world_size()
    dist.all_gather_object(lst, obj)
    return lst


def c2_parity(ex, args, params, pool):
    """--check-parity (C5 rehearsal): every pair of this rank's last timed batch
    against the CPU oracle (extract L + R + ComputeStereoMatches on the same pair, same resize
    mode): keypoints, descriptors, mvuRight and mvDepth bit-exact. After the timed region."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    nf, sf, nl, ith, mth, bf, mb = params
    kb = (args.steps - 1) % args.bufs   # c2_buffers' batch the last timed step ran on
    cache, bad = {}, []
    for i in range(args.batch):
        j = (i + 3 * kb) % len(pool)
        if j not in cache:
            L, R = pool[j]
            if kb:
                L, R = np.roll(L, 7 * kb, axis=1), np.roll(R, 7 * kb, axis=1)
            oL = oracle.Extractor(int(nf), float(sf), int(nl), int(ith), int(mth), resize_mode=args.resize_mode,
                                  blur_mode=args.blur_mode)
            oR = oracle.Extractor(int(nf), float(sf), int(nl), int(ith), int(mth), resize_mode=args.resize_mode,
                                  blur_mode=args.blur_mode)
            kL, dL = oL.extract(L)
            kR, dR = oR.extract(R)
            u, d = oracle.stereo_matches(oL, oR, kL, dL, kR, dR, float(bf), mb)
            cache[j] = (kL, dL, kR, dR, u, d)
        rkL, rdL, rkR, rdR, ru, rd = cache[j]
        gkL, gdL, gkR, gdR = ex.fetch(i)
        gu, gd = ex.stereo_fetch(i)
        n = len(rkL)
        ok = (gkL.tobytes() == rkL.tobytes() and np.array_equal(gdL, rdL) and gkR.tobytes() == rkR.tobytes()
              and np.array_equal(gdR, rdR) and gu[:n].tobytes() == ru.tobytes() and gd[:n].tobytes() == rd.tobytes())
        if not ok:
            bad.append(i)
    rank = int(os.environ.get("RANK", "0"))
    return {"rank": rank, "pairs_checked": args.batch, "pairs_bit_exact": args.batch - len(bad),
            "first_mismatch": bad[:4], "distinct_pairs": len(cache), "left_seed_first_pair": POOL_SEEDS[0],
            "resize_mode": args.resize_mode, "blur_mode": args.blur_mode}


def isolated_launch_ms(amd, params, buf, pairs, name, resize_mode=0, reps=5):
    """Average duration (hipEvents) of kernel `name` when one engine runs `pairs` stereo pairs
    of `buf` alone on the GPU (after the timed region; not part of `value`)."""
    nf, sf, nl, ith, mth, bf, mb = params
    ex1 = amd.StereoPipeline(int(nf), float(sf), int(nl), int(ith), int(mth), n_engines=1,
                             resize_mode=resize_mode)
    try:
        ex1.reserve(W, H, pairs)
        for _ in range(2):
            ex1.stereo_batch(buf.data_ptr(), pairs, W, H, W, W * H, float(bf), mb)
        amd.device_sync()
        ex1.profile(True)
        for _ in range(reps):
            ex1.stereo_batch(buf.data_ptr(), pairs, W, H, W, W * H, float(bf), mb)
            amd.device_sync()   # one launch at a time: nothing else on the GPU
        pr = ex1.profile_read()
        ex1.profile(False)
    finally:
        ex1.close()
    if name not in pr:
        return None
    tot, n = pr[name]
    return tot / n


FP64_MFMA_PEAK_TFS = 75.08   # measured, tools/microbench/mfma_f64_peak.hip (profiles/r02_mfma_f64_peak.json)


def lba_flops(prob: dict) -> dict:
    """SURVEY §8d algorithmic FP64 flops of one LM trial: E * 450 (residual, Jacobians, quadratic
    form) + sum over points of k(k+1)/2 * 324 + k * 90 + 60 (Schur pair products, k = free-pose
    observations of the point) + (6P)^3 / 3 (Cholesky)."""
    fixed = np.asarray(prob["pose_fixed"]).astype(bool)
    ep = np.asarray(prob["edge_pose"])
    free = ~fixed[ep]
    k = np.bincount(np.asarray(prob["edge_point"])[free], minlength=len(prob["point_id"])).astype(np.float64)
    P = int((~fixed).sum())
    lin = 450.0 * len(ep)
    schur = float((k * (k + 1) / 2 * 324 + k * 90 + 60).sum())
    chol = (6.0 * P) ** 3 / 3
    return {"linearize": lin, "schur": schur, "cholesky": chol, "per_trial": lin + schur + chol}


def bench_localba(amd, args, dist, world, with_cpu):
    """C4: LocalBundleAdjustment on the synthetic 20 KF x 3000 MP graph; one LocalBA call per
    inserted keyframe (LocalMapping.cc:116-118) -> keyframes/s = calls/s, summed over ranks."""
    from orbslam2_amd import synth
    from orbslam2_amd import dist as odist
    # C5: rank 0 owns the map; its snapshot (poses, points, observations) reaches every rank
    # in one RCCL broadcast over xGMI before timing
    rank = dist.get_rank() if dist is not None else 0
    prob = synth.localba_problem(seed=4) if rank == 0 else None
    prob = odist.broadcast_map(prob, COLL_DEV, dist)
    map_bytes = int(sum(a.nbytes for a in prob.values()))
    lba = amd.LocalBundleAdjustment()
    for _ in range(2):
        r = lba.solve(prob)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.lba_steps):
        r = lba.solve(prob)
    dt = time.perf_counter() - t0
    dt = odist.max_over_ranks(dt, COLL_DEV, dist)
    parity = None
    if args.check_parity:   # this rank's LocalBA on the broadcast map vs the oracle (1e-4, same LM, same erase set)
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle
        ref = oracle.lba_solve(prob)

        def rel(a, b):
            a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
            return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))
        pr, xr = rel(r["pose_Tcw"], ref["pose_Tcw"]), rel(r["point_Xw"], ref["point_Xw"])
        parity = {"rank": rank, "map_bytes": map_bytes, "pose_rel": pr, "point_rel": xr,
                  "same_lm_iterations": list(r["iterations"]) == list(ref["iterations"]),
                  "same_erase_set": bool(np.array_equal(r["edge_erase"], ref["edge_erase"])),
                  "within_1e-4": pr < 1e-4 and xr < 1e-4}
        parity = gather_ranks(parity, dist)
    res = {"localba_kf_per_s": round(world * args.lba_steps / dt, 3),
           "localba": {"ms_per_call": round(1000 * dt / args.lba_steps, 3), "edges": int(len(prob["edge_point"])),
                       "keyframes": 20, "map_points": 3000, "lm_iterations": list(r["iterations"]),
                       "lm_trials": list(r["trials"]),
                       "dtype": "f64", "lm_control": "device-resident LM state (ping-pong buffers): each trial's decision runs "
                                                     "inside the next trial's lba_reduce_points, the chunk's last in a "
                                                     "one-block lba_decide; one host readback per chunk of trials",
                       "map_snapshot_bytes": map_bytes,
                       "map_source": (f"rank 0, {'RCCL' if DIST_BACKEND == 'nccl' else DIST_BACKEND} broadcast"
                                      if dist is not None else "local")}}
    # roofline: algorithmic FP64 flops per LM trial over the measured device time of
    # one trial, against the FP64 matrix peak; the Schur SYRK alone against the same peak
    ncall = 5
    lba.profile(True)
    for _ in range(ncall):
        r = lba.solve(prob)
    prof = lba.profile_read()
    lba.profile(False)
    trials = sum(r["trials"])
    fl = lba_flops(prob)
    gpu_ms_call = sum(v[0] for v in prof.values()) / ncall
    syrk_ms, syrk_n = prof.get("lba_schur_tiles", (0.0, 1))
    syrk_avg_s = syrk_ms / max(syrk_n, 1) / 1e3
    trial_s = gpu_ms_call / 1e3 / max(trials, 1)
    achieved = fl["per_trial"] / trial_s / 1e12
    pmc, pmc_note = load_pmc_doc("lba_pmc.json", amd.build_id())
    res["localba"]["roofline"] = {
        "bound": "mfma", "kernel": "LM trial (linearize .. decide)", "achieved": round(achieved, 5),
        "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": round(achieved / FP64_MFMA_PEAK_TFS, 7), "traffic": None,
        "algorithmic_flops_per_trial": fl["per_trial"], "flops_split": fl, "trial_ms": round(trial_s * 1e3, 4),
        "schur": {"kernel": "lba_schur_tiles", "avg_launch_ms": round(syrk_avg_s * 1e3, 4),
                 "achieved": round(fl["schur"] / syrk_avg_s / 1e12, 4) if syrk_avg_s > 0 else None,
                 "frac": round(fl["schur"] / syrk_avg_s / 1e12 / FP64_MFMA_PEAK_TFS, 5) if syrk_avg_s > 0 else None},
        "peak_source": "v_mfma_f64_16x16x4_f64 measured on this MI355X (tools/microbench/mfma_f64_peak.hip; AMD spec 78.6)",
        "pmc": pmc, "pmc_source": pmc_note}
    if parity is not None:
        res["localba"]["parity_check"] = parity
    res["localba"]["gpu_ms_per_call"] = round(gpu_ms_call, 4)
    res["localba"]["host_ms_per_call"] = round(1000 * dt / args.lba_steps - gpu_ms_call, 4)
    res["localba"]["kernel_ms_per_call"] = {k: round(v[0] / ncall, 4) for k, v in sorted(prof.items())}
    if with_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 5.0:
            oracle.lba_solve(prob)
            n += 1
        cdt = time.perf_counter() - t0
        res["localba"]["cpu_baseline"] = {"value": round(n / cdt, 3), "unit": "keyframes/s", "cores": 1,
                                          "kind": "port", "sample": f"{n} LocalBA calls on the C4 graph, {cdt:.1f} s"}
    return res


def bench_rgbd(amd, args, dist, world):
    """C3: TUM-like RGB-D 640x480 stream, ORBextractor(1000) + UndistortKeyPoints +
    ComputeStereoFromRGBD + SearchForInitialization(F_t-1, F_t, 100), frames resident in HBM."""
    import torch
    from orbslam2_amd import synth
    from orbslam2_amd import dist as odist
    T = args.rgbd_batch
    K = [517.306408, 516.469215, 318.643040, 255.313989]
    D = [0.262383, -0.953104, -0.005358, 0.002628, 1.163314]
    pool = [synth.rgbd_frame(480, 640, t) for t in range(8)]
    g = torch.from_numpy(np.stack([pool[t % 8][0] for t in range(T)])).cuda()
    d = torch.from_numpy(np.stack([pool[t % 8][1] for t in range(T)])).cuda()
    torch.cuda.synchronize()
    # consecutive batches alternate over --rgbd-engines engines (one HIP stream each), so one
    # batch's latency-bound matcher overlaps the next batch's VALU-bound extraction
    exs = [amd.BatchExtractor(1000) for _ in range(max(1, args.rgbd_engines))]
    for ex in exs:
        ex.reserve(640, 480, T)

    def step(k):
        ex = exs[k % len(exs)]
        ex.extract_device(g.data_ptr(), T, 640, 480, 640, 640 * 480)
        ex.rgbd_device(d.data_ptr(), 640 * 480, 640, K, D, 40.0)
        ex.search_init_device(T - 1, 0, 1, 1, 1, K, D, 100, 0.9, True)

    for k in range(2 * len(exs)):
        step(k)
    amd.device_sync()
    t0 = time.perf_counter()
    for k in range(args.rgbd_steps):
        step(k)
    amd.device_sync()
    dt = odist.max_over_ranks(time.perf_counter() - t0, COLL_DEV, dist)
    n, m, _ = exs[(args.rgbd_steps - 1) % len(exs)].search_init_fetch(0)
    fps = world * T * args.rgbd_steps / dt
    # SURVEY §8d algorithmic bytes per RGB-D frame: gray in + keypoints / descriptors out +
    # depth gather and (uR, depth) out; HBM GB/s of that compulsory I/O against the 8 TB/s peak
    bpf = C3_BYTES_PER_FRAME
    return {"c3_rgbd_frames_per_s": round(fps, 2),
            "c3": {"frames_per_step": T, "ms_per_step": round(1000 * dt / args.rgbd_steps, 3),
                   "engines": len(exs),
                   "search_init_matches_pair0": int(n), "bytes_per_frame": bpf,
                   "hbm_gbs": round(fps / world * bpf / 1e9, 3),
                   "hbm_frac": round(fps / world * bpf / 1e9 / HBM_PEAK_GBS, 6),
                   "note": "GB/s per GPU of SURVEY §8d's compulsory bytes (640x480 u8 in, 1000 x 60 B keypoints + "
                           "descriptors out, 1000 x 12 B depth gather + uR / depth out); the rocprofv3 summary of "
                           "this leg alone is profiles/r04_kernel_stats_c3.csv (tools/gpu_c3_sweep.sh)"}}


def bench_track(amd, args, dist, world, with_cpu):
    """§8f rank 1: per-frame tracking matchers on B independent (frame, local map) problems
    resident in HBM: Frame::isInFrustum + SearchByProjection(F, vpMapPoints, th=1) (as in
    Tracking::SearchLocalPoints) + SearchByProjection(CurrentFrame, LastFrame, 15, stereo)
    (TrackWithMotionModel). 2000 keypoints, 3000 local map points, 1500 last-frame keypoints
    per frame (synth.tracking_problem)."""
    from orbslam2_amd import synth
    from orbslam2_amd import dist as odist
    B = args.track_batch
    probs = [synth.tracking_problem(300 + i, motion=("forward", "backward", "static")[i % 3]) for i in range(8)]
    t = amd.Tracker()
    t.reserve(B, 2000, 3000)
    for s in range(B):
        t.stage(s, probs[s % len(probs)])

    def step():
        t.run_local_batch(B, 0.5, 1.0, 0.8)
        t.run_frame_batch(B, 15.0, False, True)

    for _ in range(2):
        step()
    amd.device_sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.track_steps):
        step()
    amd.device_sync()
    dt = odist.max_over_ranks(time.perf_counter() - t0, COLL_DEV, dist)
    nm, _, _ = t.fetch(0, 2000)
    # ORBmatcher::Fuse(pKF, vpMapPoints, 3) search half over the same (keyframe, 3000 points)
    t.run_fuse_batch(B, 3.0)
    amd.device_sync()
    t0 = time.perf_counter()
    for _ in range(args.track_steps):
        t.run_fuse_batch(B, 3.0)
    amd.device_sync()
    fdt = odist.max_over_ranks(time.perf_counter() - t0, COLL_DEV, dist)
    res = {"track_frames_per_s": round(world * B * args.track_steps / dt, 2),
           "track": {"frames_per_step": B, "ms_per_step": round(1000 * dt / args.track_steps, 3),
                     "keypoints": 2000, "map_points": 3000, "last_keypoints": 1500,
                     "frame_matches_slot0": int(nm)},
           "fuse_keyframes_per_s": round(world * B * args.track_steps / fdt, 2)}
    t.close()
    if with_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            p = probs[n % len(probs)]
            oracle.search_local_points(p, 0.5, 1.0, 0.8)
            oracle.search_by_projection_frame(p, 15.0, False, True)
            n += 1
        cdt = time.perf_counter() - t0
        res["track"]["cpu_baseline"] = {"value": round(n / cdt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                                        "sample": f"{n} frames (8 distinct problems), oracle, single thread, {cdt:.1f} s"}
    return res


def bench_pose(amd, args, dist, world, with_cpu):
    """§8f rank 2: Optimizer::PoseOptimization on B independent frames resident in HBM
    (800 map-point matches each, 60 % stereo, 15 % outliers; synth.pose_problem), the whole
    4-round LM solve on the GPU, one workgroup per frame."""
    from orbslam2_amd import synth
    from orbslam2_amd import dist as odist
    B = args.pose_batch
    probs = [synth.pose_problem(500 + i, n=800) for i in range(8)]
    po = amd.PoseOptimizer()
    po.reserve(B, 800)
    for s in range(B):
        po.stage(s, probs[s % len(probs)])
    for _ in range(2):
        po.run_batch(B)
    amd.device_sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.pose_steps):
        po.run_batch(B)
    amd.device_sync()
    dt = odist.max_over_ranks(time.perf_counter() - t0, COLL_DEV, dist)
    r = po.fetch(0, 800)
    res = {"pose_frames_per_s": round(world * B * args.pose_steps / dt, 2),
           "pose": {"frames_per_step": B, "ms_per_step": round(1000 * dt / args.pose_steps, 3), "edges": 800,
                    "inliers_slot0": int(r["n_inliers"]), "lm_iterations_slot0": list(r["iterations"]),
                    "dtype": "f64"}}
    po.close()
    if with_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            oracle.pose_optimization(probs[n % len(probs)])
            n += 1
        cdt = time.perf_counter() - t0
        res["pose"]["cpu_baseline"] = {"value": round(n / cdt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                                       "sample": f"{n} frames (8 distinct problems), oracle, single thread, {cdt:.1f} s"}
    return res


def bench_bow(amd, args, dist, world, with_cpu):
    """§8f rank 3: Frame::ComputeBoW = DBoW2 transform(levelsup 4) of B frames x 2000
    descriptors resident in HBM against a k=10, L=6 vocabulary (1.11 M nodes, ORBvoc.txt
    shape; synthetic, synth.vocabulary)."""
    import torch
    from orbslam2_amd import synth
    from orbslam2_amd import dist as odist
    B, N = args.bow_batch, 2000
    voc = synth.vocabulary(11, 10, 6)
    feats = [synth.bow_features(voc, 700 + i, N) for i in range(8)]
    V = amd.Vocabulary(voc)
    buf = np.stack([feats[i % 8] for i in range(B)])
    d = torch.from_numpy(buf).cuda()
    c = torch.full((B,), N, dtype=torch.int32).cuda()
    torch.cuda.synchronize()

    def step():
        V.transform_batch_device(d.data_ptr(), c.data_ptr(), B, N, N * 32, 4)

    for _ in range(2):
        step()
    amd.device_sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.bow_steps):
        step()
    amd.device_sync()
    dt = odist.max_over_ranks(time.perf_counter() - t0, COLL_DEV, dist)
    r = V.batch_fetch(0, N)
    res = {"bow_frames_per_s": round(world * B * args.bow_steps / dt, 2),
           "bow": {"frames_per_step": B, "ms_per_step": round(1000 * dt / args.bow_steps, 3), "features": N,
                   "vocabulary": "k=10 L=6 (1111111 nodes)", "words_frame0": int(len(r["words"])),
                   "fv_nodes_frame0": int(len(r["fv_nodes"]))}}
    V.close()
    if with_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle
        O = oracle.Vocabulary(voc)
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            O.transform(feats[n % 8], 4)
            n += 1
        cdt = time.perf_counter() - t0
        res["bow"]["cpu_baseline"] = {"value": round(n / cdt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                                      "sample": f"{n} frames x {N} descriptors, oracle, single thread, {cdt:.1f} s"}
    return res


def bench_bowmatch(amd, args, dist, world, with_cpu):
    """§8f rank 4: ORBmatcher::SearchByBoW(KF, F) (TrackReferenceKeyFrame, nnratio 0.7) +
    SearchForTriangulation(KF1, KF2) (CreateNewMapPoints) on B keyframe pairs resident in HBM,
    2000 keypoints each (synth.bow_match_problem)."""
    from orbslam2_amd import synth
    from orbslam2_amd import dist as odist
    B = args.bowmatch_batch
    probs = [synth.bow_match_problem(900 + i, n=2000) for i in range(8)]
    m = amd.BowMatcher()
    m.reserve(B, 2000)
    for s in range(B):
        m.stage(s, probs[s % len(probs)])

    def step():
        m.run_bow_batch(B, 0.7, True)
        m.run_tri_batch(B, False, True)

    for _ in range(2):
        step()
    amd.device_sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.bowmatch_steps):
        step()
    amd.device_sync()
    dt = odist.max_over_ranks(time.perf_counter() - t0, COLL_DEV, dist)
    pairs0 = m.fetch(0, True, 2000)
    res = {"bowmatch_pairs_per_s": round(world * B * args.bowmatch_steps / dt, 2),
           "bowmatch": {"pairs_per_step": B, "ms_per_step": round(1000 * dt / args.bowmatch_steps, 3),
                        "keypoints": 2000, "triangulation_pairs_slot0": int(len(pairs0))}}
    m.close()
    if with_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            p = probs[n % len(probs)]
            oracle.search_by_bow(p, 0.7, True)
            oracle.search_for_triangulation(p)
            n += 1
        cdt = time.perf_counter() - t0
        res["bowmatch"]["cpu_baseline"] = {"value": round(n / cdt, 2), "unit": "pairs/s", "cores": 1, "kind": "port",
                                           "sample": f"{n} keyframe pairs (8 distinct), oracle, single thread, {cdt:.1f} s"}
    return res


def bench_newpts(amd, args, dist, world, with_cpu):
    """§8f rank 4: the triangulation loop of LocalMapping::CreateNewMapPoints on B (current
    keyframe, neighbour) slots resident in HBM, ~1200 SearchForTriangulation pairs each
    (synth.newpoints_problem, KITTI stereo and TUM RGB-D alternating)."""
    from orbslam2_amd import synth
    from orbslam2_amd import dist as odist
    B = args.newpts_batch
    probs = [synth.newpoints_problem(1100 + i, cam="kitti" if i % 2 == 0 else "tum") for i in range(8)]
    m = amd.NewMapPoints()
    m.reserve(B, 1500, max(len(p["pairs"]) for p in probs))
    for s in range(B):
        m.stage(s, probs[s % len(probs)])
    n_pairs = sum(len(probs[s % len(probs)]["pairs"]) for s in range(B))
    for _ in range(2):
        m.run_batch(B)
    amd.device_sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.newpts_steps):
        m.run_batch(B)
    amd.device_sync()
    dt = odist.max_over_ranks(time.perf_counter() - t0, COLL_DEV, dist)
    n0, _, _ = m.fetch(0, len(probs[0]["pairs"]))
    res = {"newpts_matches_per_s": round(world * n_pairs * args.newpts_steps / dt, 1),
           "newpts": {"slots_per_step": B, "matches_per_step": n_pairs,
                      "ms_per_step": round(1000 * dt / args.newpts_steps, 4), "new_points_slot0": int(n0),
                      "dtype": "f32 / f64 (OpenCV float Jacobi SVD with double norms)"}}
    m.close()
    if with_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle
        n = k = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            p = probs[k % len(probs)]
            oracle.triangulate(p)
            n += len(p["pairs"])
            k += 1
        cdt = time.perf_counter() - t0
        res["newpts"]["cpu_baseline"] = {"value": round(n / cdt, 1), "unit": "matches/s", "cores": 1, "kind": "port",
                                         "sample": f"{n} matches (8 distinct keyframe pairs), oracle, single thread, {cdt:.1f} s"}
    return res


def kernel_base(name: str) -> str:
    """rocprofv3 kernel name -> the engine profiler's name (template arguments dropped)."""
    return name.split("(")[0].split("<")[0].split("::")[-1]


def load_pmc_doc(fname: str, build_id: str, **expect):
    """A committed rocprofv3 PMC summary under profiles/ and whether it describes the library
    being run: its `stamp.src_hash` (tools/src_hash.py at profiling time) must equal
    orbx_build_id() of the loaded library and every `expect` key (batch, resize_mode, ...) must
    match the stamp. -> (kernels by base name or None, note)."""
    f = ROOT / "profiles" / fname
    if not f.exists():
        return None, f"profiles/{fname} absent"
    try:
        doc = json.loads(f.read_text())
    except ValueError:
        return None, f"profiles/{fname} unreadable"
    stamp = doc.get("stamp") or {}
    if stamp.get("src_hash") != build_id:
        return None, (f"profiles/{fname} was measured on library sources {stamp.get('src_hash')} "
                      f"(commit {stamp.get('commit')}), this library is {build_id}: counters not reported")
    for k, v in expect.items():
        if stamp.get(k) != v:
            return None, f"profiles/{fname} stamp {k}={stamp.get(k)}, this run {k}={v}: counters not reported"
    kern = {kernel_base(k): v for k, v in doc.get("kernels", {}).items()}
    kern["__stamp__"] = stamp
    if doc.get("step_traffic_bytes"):
        kern["__step_traffic__"] = doc["step_traffic_bytes"]
    return kern, f"profiles/{fname} (src_hash {build_id}, commit {stamp.get('commit')})"


# VALU issue ceiling: a wave64 VALU instruction occupies one 16-lane SIMD for 4 cycles;
# 256 CUs x 4 SIMDs at the 2.4 GHz peak engine clock (MI355X_MICROARCH.md)
VALU_SIMDS, VALU_CLOCK_HZ, VALU_CYCLES_PER_INST = 1024, 2.4e9, 4

# collectives: RCCL ("nccl") on device tensors; ORBSLAM_DIST_BACKEND=gloo (CPU tensors) is
# only for rehearsing the multi-rank path with several ranks sharing one GPU
DIST_BACKEND = os.environ.get("ORBSLAM_DIST_BACKEND", "nccl")
COLL_DEV = "cuda" if DIST_BACKEND == "nccl" else "cpu"


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n: int, argv, timeout_s: float, script=None) -> int:
    """`bench.py --gpus N` started as a plain process (no WORLD_SIZE in the environment): start
    `python -m torch.distributed.run --nproc-per-node N` over this script as a CHILD process, one
    rank per GPU. This process never touches the GPU (no torch import, no HIP call)
    and never execs: it relays the ranks' stderr as it comes, rank 0's JSON line on stdout, and
    returns non-zero when any rank fails (torchrun's exit status), when no JSON line arrives, or
    when the job outlives `timeout_s` (the whole process group is then killed, status 124)."""
    import signal
    import subprocess
    import threading
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(script or Path(__file__).resolve()), *argv]
    env = dict(os.environ, ORBSLAM_BENCH_LAUNCH="self", MASTER_ADDR="127.0.0.1")
    log(f"bench.py: self-launching {n} ranks: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, start_new_session=True)
    lines = []

    def pump():
        for ln in p.stdout:
            lines.append(ln.rstrip("\n"))
            if not ln.startswith("{"):
                sys.stderr.write(ln)   # the ranks' own stdout chatter goes to stderr: stdout is the line
                sys.stderr.flush()
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    try:
        rc = p.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        log(f"bench.py: ranks still running after {timeout_s:.0f} s: killing the process group")
        for sig, grace in ((signal.SIGTERM, 15), (signal.SIGKILL, 15)):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                break
            try:
                p.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        th.join(timeout=5)
        return 124
    th.join(timeout=30)
    if rc != 0:
        log(f"bench.py: torch.distributed.run exited with status {rc} (a rank failed)")
        return rc
    for ln in reversed(lines):
        if ln.startswith("{"):
            try:
                doc = json.loads(ln)
            except ValueError:
                continue
            if "metric" in doc:
                print(json.dumps(doc), flush=True)
                return 0
    log("bench.py: the ranks exited 0 but rank 0 printed no JSON line")
    return 1


def rank_topology(dist, device):
    """This rank's (rank, local rank, device, PCI bus) for `config`; every rank's when distributed."""
    import torch
    me = {"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "device": int(device)}
    try:
        pr = torch.cuda.get_device_properties(device)
        me["pci_bus_id"] = f"{getattr(pr, 'pci_domain_id', 0):04x}:{getattr(pr, 'pci_bus_id', 0):02x}:" \
                           f"{getattr(pr, 'pci_device_id', 0):02x}"
        me["name"] = pr.name
    except Exception:   # informational only
        pass
    return gather_ranks(me, dist)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Without WORLD_SIZE in the environment and N > 1, bench.py "
                         "starts torch.distributed.run with N ranks as a child process and relays rank 0's line")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launch: seconds before the ranks' process group is killed (status 124)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=384, help="stereo frames per step")
    ap.add_argument("--engines", type=int, default=3,
                    help="pipeline engines (HIP streams) the batch is split over (orbx_pipeline_*; "
                         "tools/pipeline_exp.py: 1 x 384 49.1k, 2 x 192 51.8k, 3 x 128 54.2k stereo fps)")
    ap.add_argument("--e2e-engines", type=int, default=2,
                    help="pipeline engines of the host-batch (value_e2e) leg (tools/e2e_queues.sh, 8 HW "
                         "queues: 2 engines 57.8k, 3 engines 53.0k stereo fps)")
    ap.add_argument("--pool", type=int, default=8, help="distinct synthetic stereo pairs")
    ap.add_argument("--resize-mode", type=int, default=0, choices=(0, 1),
                    help="SURVEY A.2 vertical-pass variant of the headline value (0: FixedPtCast, 1: SSE2)")
    ap.add_argument("--blur-mode", type=int, default=0, choices=(0, 1),
                    help="SURVEY A.3 GaussianBlur variant of the headline value (0: >= 3.4 fixed point, 1: 3.2 SSE2)")
    ap.add_argument("--no-alt-resize", action="store_true",
                    help="skip the alternative variant lines (other resize mode; OpenCV 3.2 resize + blur)")
    ap.add_argument("--check-parity", action="store_true",
                    help="after timing, check every rank's last C2 batch bit-exact and its LocalBA within 1e-4 "
                         "against the CPU oracle (C5 rehearsal)")
    ap.add_argument("--bufs", type=int, default=4, help="rotating resident input batches")
    ap.add_argument("--cpu-frames", type=int, default=96)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip roofline.isolated (its extra launches would enter a rocprofv3 average of the "
                         "dominant kernel: tools/gpu_trace.sh passes this so the summary matches the line)")
    ap.add_argument("--lba-steps", type=int, default=10, help="timed LocalBA calls (C4 graph)")
    ap.add_argument("--no-lba", action="store_true")
    ap.add_argument("--rgbd-batch", type=int, default=256)
    ap.add_argument("--rgbd-steps", type=int, default=40,
                    help="timed C3 batches (10 timed batches read 3-4 %% low: the pipeline fill and drain of the "
                         "engines weigh on a 11 ms region; profiles/r04_c3_sweep.log)")
    ap.add_argument("--rgbd-engines", type=int, default=4,
                    help="engines the C3 batches alternate over (one HIP stream each; round 4, 40 batches: "
                         "2: 217k, 3: 230-233k, 4: 236-237k frames/s, profiles/r04_c3_sweep.log)")
    ap.add_argument("--no-rgbd", action="store_true")
    ap.add_argument("--track-batch", type=int, default=256)
    ap.add_argument("--track-steps", type=int, default=10)
    ap.add_argument("--no-track", action="store_true")
    ap.add_argument("--pose-batch", type=int, default=256)
    ap.add_argument("--pose-steps", type=int, default=10)
    ap.add_argument("--no-pose", action="store_true")
    ap.add_argument("--bow-batch", type=int, default=256)
    ap.add_argument("--bow-steps", type=int, default=10)
    ap.add_argument("--no-bow", action="store_true")
    ap.add_argument("--bowmatch-batch", type=int, default=256)
    ap.add_argument("--bowmatch-steps", type=int, default=10)
    ap.add_argument("--no-bowmatch", action="store_true")
    ap.add_argument("--newpts-batch", type=int, default=256)
    ap.add_argument("--newpts-steps", type=int, default=10)
    ap.add_argument("--no-newpts", action="store_true")
    ap.add_argument("--latency-frames", type=int, default=512)
    ap.add_argument("--latency-warmup", type=int, default=16)
    ap.add_argument("--cpu-latency-frames", type=int, default=512)
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-c2", action="store_true", help="skip the headline leg (profiling the other legs)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:   # before anything touches the GPU: the ranks are child processes
            sys.exit(self_launch(args.gpus, sys.argv[1:], args.launch_timeout))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        ap.error(f"WORLD_SIZE={os.environ['WORLD_SIZE']} (launcher) but --gpus {args.gpus}: refusing to run a "
                 f"world size the caller did not ask for")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    ndev = torch.cuda.device_count()
    if world > 1 and DIST_BACKEND == "nccl" and ndev < int(os.environ.get("LOCAL_WORLD_SIZE", world)):
        raise SystemExit(f"bench.py: {os.environ.get('LOCAL_WORLD_SIZE', world)} ranks on this node but {ndev} "
                         f"visible GPUs: RCCL needs one GPU per rank (ORBSLAM_DIST_BACKEND=gloo rehearses several "
                         f"ranks on one GPU)")
    device = local_rank % max(ndev, 1)   # one GPU per rank (wraps only in gloo rehearsals)
    torch.cuda.set_device(device)
    torch.cuda.init()
    dist = None
    # ORBSLAM_DIST_FORCE=1: the process group (and every collective of the multi-rank path: the shared
    # parameters, the LocalBA map broadcast, the max-over-ranks timing) at world size 1 too -- the RCCL
    # path on the one GPU of a test box (tests/test_c5_rehearsal_gpu.py::test_rccl_single_rank)
    if world > 1 or os.environ.get("ORBSLAM_DIST_FORCE") == "1":
        import torch.distributed as dist
        if DIST_BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(DIST_BACKEND)
    import orbslam2_amd as amd
    amd.set_device(device)

    from orbslam2_amd import dist as odist
    B = args.batch
    # shared read-only state: ORB params + camera, broadcast once from rank 0 over RCCL
    nf, sf, nl, ith, mth, bf, fx, w, h = odist.broadcast_shared(
        [NFEAT, 1.2, 8, 20, 7, KITTI_BF, KITTI_FX, W, H] if rank == 0 else [0] * 9, COLL_DEV, dist)
    mb = float(np.float32(bf) / np.float32(fx))
    topo = rank_topology(dist, device)

    pool = make_pool(args.pool, rank, world)
    if args.no_c2:   # profiling of the other legs only (e.g. the C3 rocprofv3 summary): no headline value
        out = {"metric": "frames/sec ORB extract+match @1241x376 (1 GPU) + LocalBA keyframes/sec", "value": None,
               "unit": "stereo frames/s", "n_gpus": world, "note": "--no-c2: headline leg skipped", "config": {}}
    else:
        out = bench_c2(amd, args, dist, world, (nf, sf, nl, ith, mth, bf, mb), pool)
    out["config"].update({
        "world_size": dist.get_world_size() if dist is not None else 1,
        "dist_backend": (("rccl (torch nccl)" if DIST_BACKEND == "nccl" else DIST_BACKEND) if dist is not None
                         else None),
        "launch": ("bench.py self-launch (torch.distributed.run child)" if os.environ.get("ORBSLAM_BENCH_LAUNCH") == "self"
                   else "external torch.distributed.run" if dist is not None else "single process"),
        "rank_devices": topo})
    if not args.no_e2e and not args.no_c2:
        out.update(bench_e2e(amd, args, pool, bf, mb))
    if not args.no_latency and rank == 0:
        out.update(bench_latency(amd, args, pool, world == 1 and not args.no_cpu_baseline))
    if not args.no_rgbd:
        out.update(bench_rgbd(amd, args, dist, world))
    if not args.no_track:
        out.update(bench_track(amd, args, dist, world, rank == 0 and world == 1 and not args.no_cpu_baseline))
    if not args.no_pose:
        out.update(bench_pose(amd, args, dist, world, rank == 0 and world == 1 and not args.no_cpu_baseline))
    if not args.no_bow:
        out.update(bench_bow(amd, args, dist, world, rank == 0 and world == 1 and not args.no_cpu_baseline))
    if not args.no_bowmatch:
        out.update(bench_bowmatch(amd, args, dist, world, rank == 0 and world == 1 and not args.no_cpu_baseline))
    if not args.no_newpts:
        out.update(bench_newpts(amd, args, dist, world, rank == 0 and world == 1 and not args.no_cpu_baseline))
    if not args.no_lba:
        out.update(bench_localba(amd, args, dist, world, rank == 0 and world == 1 and not args.no_cpu_baseline))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pool, args.cpu_frames)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
