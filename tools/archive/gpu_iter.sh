#!/bin/bash
# One iteration on a kernel change: the C2-path parity tests, the pipelined C2 step and the
# isolated per-kernel profile (tools/gpu_kprof.sh). TESTS overrides the test files.
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_extract_gpu.py tests/test_stereo_gpu.py tests/test_headline_gpu.py tests/test_host_cpp_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/iter_tests.log 2>&1
rc=$?; tail -3 gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit $rc
L=orb-slam2-noted_amd/liborbslam2_amd.so
timeout -k 10 300 python tools/skip_exp.py base=$L base2=$L ${EXP_EXTRA:-} > gpurun_out/iter_exp.log 2>&1
rc=$?; cat gpurun_out/iter_exp.log | tail -1; [ $rc -eq 0 ] || exit $rc
KPROF_ENVS="${KPROF_ENVS:-base}" bash tools/gpu_kprof.sh
