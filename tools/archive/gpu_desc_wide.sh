#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}
DESC_VS='83 832' bash tools/dbg/desc_diff.sh || exit $?
L=orb-slam2-noted_amd/liborbslam2_amd.so
VARS="d82=$L:0:ORBX_DESC_V=82 d83=$L:0:ORBX_DESC_V=83 d832=$L:0:ORBX_DESC_V=832 d82b=$L:0:ORBX_DESC_V=82 d83b=$L:0:ORBX_DESC_V=83" bash tools/gpu_var_exp.sh || exit $?
ORBX_DESC_V=83 bash tools/pmc_mem.sh
