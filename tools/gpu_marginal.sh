#!/bin/bash
# Marginal cost of each C2 extraction kernel inside the 3-engine pipeline: the kernel launched
# twice (ORBX_EXP_TWICE bit mask, idempotent kernels) against the base library.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
L=orb-slam2-noted_amd/liborbslam2_amd.so
timeout -k 10 500 python tools/skip_exp.py base=$L resize2=$L:1 qt2=$L:2 desc2=$L:4 stereo2=$L:8 base2=$L > gpurun_out/marginal.log 2>&1
rc=$?; cat gpurun_out/marginal.log; exit $rc
