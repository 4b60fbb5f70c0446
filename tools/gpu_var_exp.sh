#!/bin/bash
# pipelined C2 step of variant libraries / knobs (VARS: name=lib[:mask[:VAR=v,...]] ...)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
timeout -k 10 500 python tools/skip_exp.py $VARS > gpurun_out/var_exp.log 2>&1
rc=$?; cat gpurun_out/var_exp.log | tail -1; exit $rc
