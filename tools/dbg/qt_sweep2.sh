#!/bin/bash
# C2 under quadtree LDS sizes (keys in LDS per workgroup): occupancy vs keys spilled to global
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--no-e2e --no-latency --no-profile" bash tools/env_sweep.sh "X=0" "ORBX_QT_LDS_KB=24" "ORBX_QT_LDS_KB=20" "ORBX_QT_LDS_KB=32" "X=0" "ORBX_QT_LDS_KB=24" "ORBX_QT_LDS_KB=20"
