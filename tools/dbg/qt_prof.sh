#!/bin/bash
# quadtree phase clocks of an ORBX_QT_PROFILE build (orb-slam2-noted_amd/build/exp_qtprof)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
ORBSLAM_AMD_LIB=orb-slam2-noted_amd/build/exp_qtprof/liborbslam2_amd.so timeout -k 10 200 python3 tools/dbg/qt_prof.py > gpurun_out/qt_prof.log 2>&1
