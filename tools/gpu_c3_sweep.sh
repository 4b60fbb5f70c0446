#!/bin/bash
# C3 (RGB-D) leg alone over timed-region lengths and engine counts (pipeline fill / drain against
# steady state), then a rocprofv3 --kernel-trace --stats of the default configuration:
#   tools/gpu_c3_sweep.sh  -> gpurun_out/c3_sweep.log, gpurun_out/c3prof/
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
ARGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --no-e2e"
cd "$R"
for rep in 1 2; do
  for cfg in "10 3" "40 3" "40 2" "40 4" "80 3"; do
    set -- $cfg
    line=$(timeout -k 10 180 python3 bench.py $ARGS --rgbd-steps "$1" --rgbd-engines "$2" 2>/dev/null | tail -1) || exit $?
    echo "steps=$1 engines=$2 $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); print(d["c3_rgbd_frames_per_s"], d["c3"]["ms_per_step"])' "$line")" | tee -a "$OUT/c3_sweep.log"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3prof" -o run -- python3 "$R/bench.py" $ARGS --rgbd-steps 40 > "$OUT/c3_bench.json" 2> "$OUT/c3_prof.err"
rc=$?; echo "c3 prof rc=$rc"; exit $rc
