"""Marginal cost of each part of the C2 step (experiment, not a parity path): the bench's C2
pipeline (3 engines x 128 pairs, 384 pairs per step) timed with instrumented builds of the same
sources in which one part is compiled out (make variant VDEFS=-D...: FB_SKIP_PRE / FB_SKIP_EXACT /
FB_SKIP_BLUR; EXP_SKIP_RESIZE and EXP_SKIP_BRIEF were removed in round 6; outputs of a skipped part are
garbage and downstream work may change with them, so only skips whose outputs feed nothing
but pixel values are clean), or with an idempotent kernel launched twice (lib:mask ->
ORBX_EXP_TWICE=mask, orb_engine.h: the clean way to read a kernel's marginal cost). One
subprocess per run:
    python tools/skip_exp.py base=orb-slam2-noted_amd/liborbslam2_amd.so rz2=orb-slam2-noted_amd/liborbslam2_amd.so:1 ..."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

CHILD = r'''
import sys, time, json
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch
torch.cuda.init()
import orbslam2_amd as amd
from orbslam2_amd import synth
import os
W, H, B, K = 1241, 376, int(os.environ.get("EXP_B", "384")), int(os.environ.get("EXP_ENGINES", "3"))
pool = [synth.stereo_pair(H, W, t) for t in range(8)]
bufs = [torch.from_numpy(np.stack([im for i in range(B) for im in pool[(i + 3 * k) % 8]])).cuda() for k in range(2)]
mb = float(np.float32(386.1448) / np.float32(718.856))
pl = amd.StereoPipeline(2000, n_engines=K)
pl.reserve(W, H, B)
def step(k):
    pl.stereo_batch(bufs[k % 2].data_ptr(), B, W, H, W, W * H, 386.1448, mb)
best = None
for rep in range(3):
    for k in range(3):
        step(k)
    amd.device_sync()
    t0 = time.perf_counter()
    for k in range(20):
        step(k)
    amd.device_sync()
    dt = time.perf_counter() - t0
    best = dt if best is None else min(best, dt)
print(json.dumps({"fps": round(B * 20 / best, 1), "ms_per_step": round(1000 * best / 20, 4)}))
'''

if __name__ == "__main__":
    res = {}
    for arg in sys.argv[1:]:
        name, lib = arg.split("=", 1)
        twice, extra = "0", {}
        if ":" in lib:   # lib:mask[:VAR=v,VAR=v] -> ORBX_EXP_TWICE=mask (kernels launched twice) + env
            parts = lib.split(":")
            lib, twice = parts[0], parts[1] or "0"
            if len(parts) > 2:
                extra = dict(kv.split("=", 1) for kv in parts[2].split(",") if kv)
        env = dict(os.environ, ORBSLAM_AMD_LIB=str((ROOT / lib).resolve()), ORBX_EXP_TWICE=twice, **extra)
        r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT / "orb-slam2-noted_amd" / "python")], env=env,
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            res[name] = {"error": r.stderr[-800:]}
            print(name, res[name], flush=True)
            break
        res[name] = json.loads(r.stdout.strip().splitlines()[-1])
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(res))
