#!/bin/bash
# describe variants: parity of the extraction tests, then the C2 pipeline step per variant
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py tests/test_headline_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/desc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/desc_tests.log; [ $rc -eq 0 ] || exit $rc
L=orb-slam2-noted_amd/liborbslam2_amd.so
timeout -k 10 500 python tools/skip_exp.py old3=$L:0:ORBX_DESC_V=0 v82=$L:0:ORBX_DESC_V=82 v62=$L:0:ORBX_DESC_V=62 v84=$L:0:ORBX_DESC_V=84 v42=$L:0:ORBX_DESC_V=42 old3b=$L:0:ORBX_DESC_V=0 > gpurun_out/desc_exp.log 2>&1
rc=$?; cat gpurun_out/desc_exp.log; exit $rc
