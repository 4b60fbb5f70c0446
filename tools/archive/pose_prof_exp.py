import sys, time
sys.path.insert(0, 'orb-slam2-noted_amd/python')
import orbslam2_amd as amd
from orbslam2_amd import synth
po = amd.PoseOptimizer()
p = synth.pose_problem(500, n=800)
po.reserve(256, 800)
for s in range(256): po.stage(s, p)
for B in (1, 1, 256):
    amd.device_sync(); t = time.perf_counter(); po.run_batch(B); amd.device_sync(); print("B", B, (time.perf_counter() - t) * 1e3, "ms", flush=True)
