"""LocalBA beside the extraction (ADVICE r5 on lba_finish_chol): the reference runs LocalBundleAdjustment
on the LocalMapping thread while Tracking extracts every frame, so a LocalBA trial's kernels share the
GPU with the extraction engines. For each LocalBA finish path (fused lba_finish_chol: its finish blocks
and Cholesky block each need an almost empty CU -- 1024 threads and the Cholesky's LDS; two-launch:
lba_schur_finish + lba_chol_tiled), alternating: LocalBA calls on the C4 graph alone, then the same
calls on a second host thread while the main thread keeps the C2 pipeline (3 engines x 128 pairs)
busy; reports LocalBA ms per call and the C2 rate in each setting.
    python tools/lba_concurrent.py [rounds]"""
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
sys.path.insert(0, str(ROOT))
from orbslam2_amd import synth  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    # the stream first: its worker processes must not inherit or open the GPU
    pool = synth.stereo_stream(376, 1241, 512)
    import bench  # GPU_MAX_HW_QUEUES as bench.py sets it, before the runtime starts
    import torch
    torch.cuda.init()
    import orbslam2_amd as amd
    buf = bench.c2_stream_buffer(pool)
    mb = float(np.float32(386.1448) / np.float32(718.856))
    B = 384
    ex = amd.StereoPipeline(2000, 1.2, 8, 20, 7, n_engines=3)
    ex.reserve(1241, 376, B)
    prob = synth.localba_problem(seed=4)
    lba = amd.LocalBundleAdjustment()
    for _ in range(3):
        lba.solve(prob)
    N = 40


    def lba_calls(out):
        t0 = time.perf_counter()
        for _ in range(N):
            lba.solve(prob)
        out.append((time.perf_counter() - t0) / N)


    def c2_until(flag, counter):
        k = 0
        while not flag.is_set():
            ex.stereo_batch(bench.c2_batch_ptr(buf, 512, B, k), B, 1241, 376, 1241, 1241 * 376, 386.1448, mb)
            k += 1
            if k % 4 == 0:
                amd.device_sync()
        amd.device_sync()
        counter.append(k)


    res = []
    settings = [(1, 0), (0, 0), (1, 1)]   # (fused finish, high stream priority)
    for r in range(rounds):
        for fused, prio in settings:
            lba.set_test_option(lba.LBA_OPT_FUSE_FINISH, fused)
            lba.set_test_option(lba.LBA_OPT_STREAM_PRIORITY, prio)
            alone = []
            lba_calls(alone)
            both, cnt, flag = [], [], threading.Event()
            th = threading.Thread(target=c2_until, args=(flag, cnt))
            t0 = time.perf_counter()
            th.start()
            time.sleep(0.05)   # the pipeline running before the first LocalBA call
            lba_calls(both)
            flag.set()
            th.join()
            el = time.perf_counter() - t0
            row = {"round": r, "fused": fused, "high_priority": prio, "lba_ms_alone": round(alone[0] * 1e3, 4),
                   "lba_ms_beside_c2": round(both[0] * 1e3, 4), "c2_frames_per_s_beside_lba": round(cnt[0] * B / el, 1)}
            res.append(row)
            print(json.dumps(row), flush=True)
    lba.set_test_option(lba.LBA_OPT_FUSE_FINISH, 1)
    for fused, prio in settings:
        sel = [x for x in res if x["fused"] == fused and x["high_priority"] == prio]
        print("SUMMARY fused=%d high_priority=%d lba alone %.4f ms, beside C2 %.4f ms, C2 %.0f frames/s" % (
            fused, prio, np.mean([x["lba_ms_alone"] for x in sel]), np.mean([x["lba_ms_beside_c2"] for x in sel]),
            np.mean([x["c2_frames_per_s_beside_lba"] for x in sel])))


if __name__ == "__main__":   # synth.stereo_stream spawns worker processes
    main()
