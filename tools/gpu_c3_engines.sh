#!/bin/bash
# C3 leg alone at 4, 5 and 6 engines (40 timed batches), alternating, 2 rounds -> gpurun_out/c3_engines.log
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
ARGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --no-e2e --rgbd-steps 40"
for rep in 1 2; do
  for e in 4 5 6; do
    line=$(timeout -k 10 180 python3 bench.py $ARGS --rgbd-engines $e 2>/dev/null | tail -1) || exit $?
    echo "engines=$e $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); print(d["c3_rgbd_frames_per_s"], d["c3"]["ms_per_step"])' "$line")" | tee -a "$OUT/c3_engines.log"
  done
done
