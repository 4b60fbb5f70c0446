#!/bin/bash
# C2 leg alone over timed-region lengths (pipeline fill / drain against steady state):
#   tools/gpu_c2_steps.sh  -> gpurun_out/c2_steps.log
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
ARGS="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize --no-profile"
cd "$R"
for rep in 1 2; do
  for st in 20 60 120; do
    line=$(timeout -k 10 180 python3 bench.py $ARGS --steps "$st" --warmup 3 2>/dev/null | tail -1) || exit $?
    echo "steps=$st $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); print(d["value"], d["ms_per_step"])' "$line")" | tee -a "$OUT/c2_steps.log"
  done
done
