"""Experiment: two engines on two streams with their VALU-bound phase 1 (pyramid + FAST map +
blur) alternating, so one engine's phase 1 overlaps the other's latency-bound phase 2 + stereo.
Prints stereo frames/s for the plain single-engine batch and the interleaved pair."""
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


def imgs_for(B):
    return torch.from_numpy(np.stack([im for i in range(B) for im in pool[i % 4]])).cuda()


def plain(B, steps=20):
    d = imgs_for(B)
    ex = amd.BatchExtractor(2000)
    ex.reserve(W, H, 2 * B)

    def step():
        ex.extract_device(d.data_ptr(), 2 * B, W, H, W, W * H)
        ex.stereo_batch(B, 386.1448, mb)
    return timeit(step, B, steps)


def interleaved(B, steps=20, mode="alt", k=2):
    per = B // k
    d = imgs_for(B)
    exs = [amd.BatchExtractor(2000) for _ in range(k)]
    for ex in exs:
        ex.reserve(W, H, 2 * per)
    ss = [torch.cuda.ExternalStream(ex.stream()) for ex in exs]
    last = [None]

    def step():
        for j in range(k):
            ex, s = exs[j], ss[j]
            ptr = d.data_ptr() + j * 2 * per * W * H
            if mode == "alt" and last[0] is not None:
                s.wait_event(last[0])   # phase 1 after the previous engine's phase 1
            ex.extract_device_phase(ptr, 2 * per, W, H, W, W * H, 1)
            e = torch.cuda.Event()
            e.record(s)
            last[0] = e
            ex.extract_device_phase(ptr, 2 * per, W, H, W, W * H, 2)
            ex.stereo_batch(per, 386.1448, mb)
    return timeit(step, B, steps)


def timeit(step, B, steps):
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    amd.device_sync()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    amd.device_sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    return B * steps / dt, 1000 * dt / steps


cases = [tuple(int(v) if v.isdigit() else v for v in c.split(",")) for c in sys.argv[1:]] or [(256, 1, "plain"), (256, 2, "alt")]
for B, k, mode in cases:
    fps, ms = plain(B) if k == 1 else interleaved(B, mode=mode, k=k)
    print(f"B={B} engines={k} {mode}: {fps:.0f} stereo fps ({ms:.3f} ms/step)", flush=True)
