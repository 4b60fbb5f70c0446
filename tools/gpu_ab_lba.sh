#!/bin/bash
# LocalBA parity tests of the working-tree library, then a same-box A/B of the LocalBA leg against a
# baseline build, then the host-phase profile:  tools/gpu_ab_lba.sh <baseline lib.so>
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
BASE=$1
NEW="$R/orb-slam2-noted_amd/liborbslam2_amd.so"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py tests/test_host_cpp_gpu.py tests/test_c5_rehearsal_gpu.py -x -q --timeout 300 --timeout-method thread > "$OUT/ab_lba_tests.log" 2>&1
rc=$?; tail -2 "$OUT/ab_lba_tests.log"; [ $rc -eq 0 ] || exit $rc
LEGS="--no-c2 --no-cpu-baseline --no-profile --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --steps 1 --warmup 1 --lba-steps 40"
bash tools/ab_bench.sh "$BASE" "$NEW" 4 $LEGS > "$OUT/ab_lba.log" 2>&1 || exit $?
python3 - "$OUT/ab_lba.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag, js = line.split(' ', 1)
    l = json.loads(js)["localba"]
    print(tag, l["ms_per_call"], l["gpu_ms_per_call"], l["host_ms_per_call"], l["lm_trials"])
PY
ORBX_LBA_HOSTPROF=1 timeout -k 10 120 python3 tools/lba_prof.py 20 > "$OUT/lba_hostprof.txt" 2>&1; tail -3 "$OUT/lba_hostprof.txt"
