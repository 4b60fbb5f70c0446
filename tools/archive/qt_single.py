import sys
sys.path.insert(0, "orb-slam2-noted_amd/python")
import torch; torch.cuda.init()
import orbslam2_amd as amd
from orbslam2_amd import synth
L, R = synth.stereo_pair(376, 1241, 0)
ex = amd.ORBextractor(2000)
for _ in range(3): ex(L)
amd.device_sync()
