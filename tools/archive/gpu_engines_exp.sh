#!/bin/bash
# C2 pipeline step against the number of extraction engines (skip_exp's EXP_ENGINES)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
L=orb-slam2-noted_amd/liborbslam2_amd.so
timeout -k 10 500 python tools/skip_exp.py e3=$L:0:EXP_ENGINES=3 e2=$L:0:EXP_ENGINES=2 e4=$L:0:EXP_ENGINES=4 e6=$L:0:EXP_ENGINES=6 e3b=$L:0:EXP_ENGINES=3 > gpurun_out/engines.log 2>&1
rc=$?; cat gpurun_out/engines.log; exit $rc
