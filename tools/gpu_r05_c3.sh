#!/bin/bash
# C3 parity tests of the working-tree library (every SearchForInitialization path), then a same-box
# A/B of the C3 leg against a variant build ($1 = variant name), 4 rounds each.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
VAR="$R/orb-slam2-noted_amd/build/var_$1/liborbslam2_amd.so"
timeout -k 10 600 python -u -m pytest tests/test_rgbd_gpu.py tests/test_matcher_gpu.py tests/test_host_cpp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/r05_c3_tests_$1.log" 2>&1
rc=$?; tail -2 "$O/r05_c3_tests_$1.log"; [ $rc -eq 0 ] || exit $rc
LEGS="--no-c2 --no-cpu-baseline --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --steps 1 --warmup 1"
timeout -k 10 600 bash tools/ab_bench.sh "$VAR" "$R/orb-slam2-noted_amd/liborbslam2_amd.so" 4 $LEGS > "$O/r05_ab_c3_$1.log" 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$O/r05_ab_c3_$1.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag, js = line.split(' ', 1)
    d = json.loads(js)
    print(tag, d["c3_rgbd_frames_per_s"], d["c3"]["ms_per_step"], d["c3"]["search_init_matches_pair0"])
PY
