#!/bin/bash
# kernel + memory-copy trace of the C2 e2e (host-batch) leg: bench with C2 + e2e only, few steps
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/e2e_trace" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-profile --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency > "$R/gpurun_out/e2e_trace.json" 2> "$R/gpurun_out/e2e_trace.err"
rc=$?; cat "$R/gpurun_out/e2e_trace.json"; ls "$R/gpurun_out/e2e_trace"; exit $rc
