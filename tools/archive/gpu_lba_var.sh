#!/bin/bash
# LocalBA variant libraries: parity tests and wall per call (LBA_VARS: name=lib ...)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for nv in $LBA_VARS; do
  n=${nv%%=*}; lib=${nv#*=}
  ORBSLAM_AMD_LIB="$R/$lib" timeout -k 10 200 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/lbav_$n.log 2>&1
  rc=$?; echo "$n tests: $(tail -1 gpurun_out/lbav_$n.log)"; [ $rc -eq 0 ] || exit $rc
  echo "$n $(ORBSLAM_AMD_LIB="$R/$lib" timeout -k 10 120 python tools/lba_prof.py 40 2>/dev/null | tail -1)" || exit $?
done
