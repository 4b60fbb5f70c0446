"""Debug: descriptor rows of the HIP extractor against the oracle on one KITTI image, per
describe variant (ORBX_DESC_V in the environment)."""
import os
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
sys.path.insert(0, str(ROOT / "oracle"))
import torch  # noqa
torch.cuda.init()
import orbslam2_amd as amd
import oracle
from orbslam2_amd import synth
img = synth.textured_image(376, 1241, 2)
k, d = amd.ORBextractor(2000)(img)
rk, rd = oracle.Extractor(2000).extract(img)
print("variant", os.environ.get("ORBX_DESC_V"), "n", len(k), len(rk))
bad = np.nonzero((d != rd).any(axis=1))[0]
print("bad rows", len(bad), bad[:40])
for i in bad[:6]:
    g64 = d[i].view(np.uint64); r64 = rd[i].view(np.uint64)
    nb = [bin(int(a) ^ int(b)).count("1") for a, b in zip(g64, r64)]
    print(i, "octave", k[i]["octave"], "angle", k[i]["angle"], "bitdiff per word", nb,
          "gpu", [hex(int(x)) for x in g64], "ref", [hex(int(x)) for x in r64])
# does a bad GPU row equal some other oracle row / word?
rw = {int(x): j for j, row in enumerate(rd) for x in row.view(np.uint64)}
hits = sum(1 for i in bad[:200] for x in d[i].view(np.uint64) if int(x) in rw)
print("bad-row words found elsewhere in the oracle", hits, "of", 4 * min(200, len(bad)))
