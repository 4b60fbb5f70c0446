#!/bin/bash
# C2 pipeline engine count / batch sweep, same box:  tools/gpu_engines_sweep.sh -> gpurun_out/engines_sweep.log
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
C2="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize --steps 30"
for rep in 1 2; do
  for cfg in "3 384" "4 384" "4 512" "2 384" "6 384" "5 640"; do
    set -- $cfg
    line=$(timeout -k 10 180 python3 bench.py $C2 --engines "$1" --batch "$2" 2>/dev/null | tail -1) || exit $?
    echo "engines=$1 batch=$2 $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' "$line")" | tee -a "$OUT/engines_sweep.log"
  done
done
