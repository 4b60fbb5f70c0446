#!/bin/bash
# Parity tests of the working-tree library, then same-box A/B against a baseline build on the C2
# and C3 legs, then the C2 timed-region sweep:
#   tools/gpu_ab_edge.sh <baseline lib.so> "<pytest files>"
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
BASE=$1; TESTS=$2
NEW="$R/orb-slam2-noted_amd/liborbslam2_amd.so"
cd "$R"
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > "$OUT/ab_tests.log" 2>&1
rc=$?; tail -2 "$OUT/ab_tests.log"; [ $rc -eq 0 ] || exit $rc
C2="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize --no-profile --steps 40"
C3="--no-c2 --no-cpu-baseline --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency"
bash tools/ab_bench.sh "$BASE" "$NEW" 3 $C2 > "$OUT/ab_c2.log" 2>&1 || exit $?
echo "ab c2 done"
bash tools/ab_bench.sh "$BASE" "$NEW" 3 $C3 > "$OUT/ab_c3.log" 2>&1 || exit $?
echo "ab c3 done"
bash tools/gpu_c2_steps.sh || exit $?
echo "all done"
