#!/bin/bash
# LocalBA parity tests of the working-tree library, then a same-box A/B of the LocalBA leg against a
# variant build ($1 = variant name under orb-slam2-noted_amd/build/var_<name>), 4 rounds each.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
VAR="$R/orb-slam2-noted_amd/build/var_$1/liborbslam2_amd.so"
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py tests/test_host_cpp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/r05_lba_tests_$1.log" 2>&1
rc=$?; tail -2 "$O/r05_lba_tests_$1.log"; [ $rc -eq 0 ] || exit $rc
LEGS="--no-c2 --no-cpu-baseline --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --steps 1 --warmup 1 --lba-steps 40"
timeout -k 10 600 bash tools/ab_bench.sh "$VAR" "$R/orb-slam2-noted_amd/liborbslam2_amd.so" 4 $LEGS > "$O/r05_ab_lba_$1.log" 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$O/r05_ab_lba_$1.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag, js = line.split(' ', 1)
    l = json.loads(js)["localba"]
    print(tag, l["ms_per_call"], l["gpu_ms_per_call"], l["host_ms_per_call"], json.dumps(l["kernel_ms_per_call"]))
PY
