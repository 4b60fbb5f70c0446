#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C3 leg alone at the default configuration (4 engines, 40 batches)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
ARGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --no-e2e"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3prof" -o run -- python3 "$R/bench.py" $ARGS --rgbd-steps 40 > "$OUT/c3_bench.json" 2> "$OUT/c3_prof.err"
rc=$?; echo "c3 prof rc=$rc"; exit $rc
