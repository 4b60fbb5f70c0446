#!/bin/bash
# rocprofv3 kernel trace + stats of a C2-only bench (no CPU baseline); summary by tools/trace_summary.py
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/trace" -o run -- python3 "$R/bench.py" --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-isolated ${BENCH_ARGS:-} > "$R/gpurun_out/trace_bench.json" 2> "$R/gpurun_out/trace.err"
rc=$?; cat "$R/gpurun_out/trace_bench.json"; exit $rc
