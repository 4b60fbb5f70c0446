#!/bin/bash
# quadtree phase clocks (ORBX_QT_PROFILE build) and a C2 sweep of the quadtree layout knobs
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
ORBSLAM_AMD_LIB=orb-slam2-noted_amd/build/exp_qtprof/liborbslam2_amd.so timeout -k 10 200 python3 tools/dbg/qt_prof.py > gpurun_out/qt_prof.log 2>&1 || exit $?
echo "qtprof rc=0"
BENCH_ARGS="--no-e2e --no-latency --no-profile" bash tools/env_sweep.sh "X=0" "ORBX_QT_NODES_LDS=1 ORBX_QT_LDS_KB=64" "ORBX_QT_NODES_LDS=1 ORBX_QT_LDS_KB=96" "X=0" "ORBX_QT_NODES_LDS=1 ORBX_QT_LDS_KB=64" "ORBX_QT_LDS_KB=40"
