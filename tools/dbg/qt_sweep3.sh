#!/bin/bash
# C2 under quadtree LDS sizes after the level-major dispatch order
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--no-e2e --no-latency --no-profile" bash tools/env_sweep.sh "X=0" "ORBX_QT_LDS_KB=40" "ORBX_QT_LDS_KB=32" "ORBX_QT_LDS_KB=24" "X=0" "ORBX_QT_LDS_KB=40" "ORBX_QT_LDS_KB=32"
