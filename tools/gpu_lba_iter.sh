#!/bin/bash
# LocalBA iteration: parity tests, wall per call, Cholesky phase profile of the variants
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py tests/test_host_cpp_gpu.py tests/test_pose_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/lba_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lba_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/lba_prof.py 30 || exit $?
for v in ${VARIANTS-lbaprof}; do
  ORBSLAM_AMD_LIB="$R/orb-slam2-noted_amd/build/var_$v/liborbslam2_amd.so" timeout -k 10 120 python tools/lba_prof.py 3 > gpurun_out/lba_$v.txt 2>&1 || exit $?
  echo "$v $(grep LBAPROF gpurun_out/lba_$v.txt | tail -1)"
done
