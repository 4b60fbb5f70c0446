#!/bin/bash
# C3 (RGB-D) batch size x engines sweep, same box:  tools/gpu_c3_batch.sh -> gpurun_out/c3_batch.log
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
ARGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --no-e2e --rgbd-steps 40"
cd "$R"
for rep in 1 2; do
  for cfg in "256 4" "512 4" "512 3" "512 2" "768 3" "1024 2"; do
    set -- $cfg
    line=$(timeout -k 10 180 python3 bench.py $ARGS --rgbd-batch "$1" --rgbd-engines "$2" 2>/dev/null | tail -1) || exit $?
    echo "batch=$1 engines=$2 $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); print(d["c3_rgbd_frames_per_s"], d["c3"]["ms_per_step"])' "$line")" | tee -a "$OUT/c3_batch.log"
  done
done
