"""LocalBA C4 profiling driver (or a larger window: [calls seed n_kf n_points]): N calls of LocalBundleAdjustment on the synthetic 20 KF x 3000 MP
graph (bench.py's localba leg without the rest), wall time per call. Run under rocprofv3
--kernel-trace --stats (per-kernel device time) or --pmc (MFMA counters).
    python tools/lba_prof.py [calls]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
import orbslam2_amd as amd  # noqa: E402
from orbslam2_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
# optional: seed n_kf n_points (a larger window, e.g. 12 64 6000)
prob = synth.localba_problem(*(int(a) for a in sys.argv[2:5])) if len(sys.argv) > 4 else synth.localba_problem(seed=4)
lba = amd.LocalBundleAdjustment()
for _ in range(2):
    r = lba.solve(prob)
t = []
for _ in range(n):
    t0 = time.perf_counter()
    r = lba.solve(prob)
    t.append(time.perf_counter() - t0)
t.sort()
print(json.dumps({"calls": n, "median_ms": round(1000 * t[n // 2], 4), "mean_ms": round(1000 * sum(t) / n, 4),
                  "lm_iterations": list(r["iterations"]), "edges": len(prob["edge_point"])}))
