#!/bin/bash
# Round-6 LocalBA session: the LocalBA GPU tests (parity at 8..100 free keyframes, stop hooks, fused /
# two-launch bit identity, hand-off fault), then the LocalBA legs of bench.py (C4 + localba_windows).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
TAG="${TAG:-r06_lba}"
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/${TAG}_tests.log" 2>&1
rc=$?; echo "lba tests rc=$rc"; tail -4 "$O/${TAG}_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency \
  --no-cpu-baseline --steps 5 > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo done
