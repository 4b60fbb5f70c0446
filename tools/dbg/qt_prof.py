"""quadtree_kernel phase clocks (an ORBX_QT_PROFILE build, ORBSLAM_AMD_LIB): one 64-image KITTI batch
through BatchExtractor, the kernel's QTPROF printf lines summarised per level (wall_clock64 ticks).
  ORBSLAM_AMD_LIB=<profile build> python tools/dbg/qt_prof.py > log"""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
import torch
torch.cuda.init()
import orbslam2_amd as amd
from orbslam2_amd import synth
imgs = np.stack([synth.stereo_pair(376, 1241, t)[0] for t in range(64)])
d = torch.from_numpy(imgs).cuda()
ex = amd.BatchExtractor(2000)
ex.reserve(1241, 376, 64)
for _ in range(3):
    ex.extract_device(d.data_ptr(), 64, 1241, 376, 1241, 1241 * 376)
amd.device_sync()
print("done", flush=True)
