#!/bin/bash
# C2 with the quadtree node arrays in LDS after the level-major dispatch order
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--no-e2e --no-latency --no-profile" bash tools/env_sweep.sh "X=0" "ORBX_QT_NODES_LDS=1 ORBX_QT_LDS_KB=64" "ORBX_QT_NODES_LDS=1 ORBX_QT_LDS_KB=80" "X=0" "ORBX_QT_NODES_LDS=1 ORBX_QT_LDS_KB=64"
