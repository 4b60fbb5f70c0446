"""Minimal extraction loop for rocprofv3 counter passes (one batch, a few steps)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
import torch  # noqa: E402

torch.cuda.init()
import orbslam2_amd as amd  # noqa: E402
from orbslam2_amd import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
pool = [synth.stereo_pair(376, 1241, t) for t in range(4)]
imgs = np.stack([im for i in range(B) for im in pool[i % 4]])
d = torch.from_numpy(imgs).cuda()
torch.cuda.synchronize()
ex = amd.BatchExtractor(2000)
ex.reserve(1241, 376, 2 * B)
mb = float(np.float32(386.1448) / np.float32(718.856))
for _ in range(steps):
    ex.extract_device(d.data_ptr(), 2 * B, 1241, 376, 1241, 1241 * 376)
    ex.stereo_batch(B, 386.1448, mb)
amd.device_sync()
print("done")
