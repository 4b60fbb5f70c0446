"""Experiment: does splitting the C2 batch over concurrent engines (one HIP stream each) fill
the kernel tails? Prints stereo frames/s for 1 engine x B and k engines x B/k."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
import torch  # noqa: E402

torch.cuda.init()
import orbslam2_amd as amd  # noqa: E402
from orbslam2_amd import synth  # noqa: E402

W, H = 1241, 376
pool = [synth.stereo_pair(H, W, t) for t in range(4)]
mb = float(np.float32(386.1448) / np.float32(718.856))


def run(B, k, steps=10):
    imgs = np.stack([im for i in range(B) for im in pool[i % 4]])
    d = torch.from_numpy(imgs).cuda()
    torch.cuda.synchronize()
    per = B // k
    exs = []
    for j in range(k):
        ex = amd.BatchExtractor(2000)
        ex.reserve(W, H, 2 * per)
        exs.append(ex)

    def step():
        for j, ex in enumerate(exs):
            ex.extract_device(d.data_ptr() + j * 2 * per * W * H, 2 * per, W, H, W, W * H)
            ex.stereo_batch(per, 386.1448, mb)

    for _ in range(3):
        step()
    amd.device_sync()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    amd.device_sync()
    dt = time.perf_counter() - t
    print(f"B={B} engines={k}: {B * steps / dt:.0f} stereo fps ({1000 * dt / steps:.3f} ms/step)", flush=True)


for B, k in [(128, 1), (128, 2), (128, 4), (256, 1), (256, 2), (64, 1), (512, 2)]:
    run(B, k)
