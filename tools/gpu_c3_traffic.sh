#!/bin/bash
# L2 -> fabric bytes of the C3 (RGB-D) leg alone, per kernel launch (request-size counters,
# tools/pmc_reqsize.sh) -> gpurun_out/c3_traffic.json
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"
ARGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --no-e2e --rgbd-steps 8"
bash "$R/tools/pmc_reqsize.sh" c3 python3 "$R/bench.py" $ARGS || exit $?
python3 "$R/tools/reqsize_summary.py" "$O" c3 > "$O/c3_traffic.json"; rc=$?; echo "summary rc=$rc"; exit $rc
