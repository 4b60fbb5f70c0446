"""Debug: keypoints that differ between the HIP extractor and the oracle on one KITTI image."""
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
ex = oracle.Extractor(2000)
rk, rd = ex.extract(img)
print("gpu", len(k), "oracle", len(rk))
g = {(int(a["octave"]), float(a["x"]), float(a["y"])): float(a["response"]) for a in k}
r = {(int(a["octave"]), float(a["x"]), float(a["y"])): float(a["response"]) for a in rk}
only_g = sorted(set(g) - set(r)); only_r = sorted(set(r) - set(g))
print("only gpu", len(only_g), only_g[:20])
print("only oracle", len(only_r), only_r[:20])
for key in only_g[:5] + only_r[:5]:
    print(key, g.get(key), r.get(key))
# per level candidates: compare the level's FAST scores at the differing points
for (l, x, y) in (only_g + only_r)[:10]:
    s = ex.s.mvScaleFactor[l]
    px, py = (x / s, y / s) if l else (x, y)
    lev = ex.level(l)
    xi, yi = int(round(px)), int(round(py))
    print("level", l, "pix", xi, yi, "val", lev[yi, xi])
