#!/bin/bash
# in-kernel Cholesky phase split (LBA_PROFILE) of the builds build/var_lbaprof_<name> named in $@
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
for v in "$@"; do
  ORBSLAM_AMD_LIB="$R/orb-slam2-noted_amd/build/var_lbaprof_$v/liborbslam2_amd.so" timeout -k 10 120 python3 tools/lba_prof.py 2 > "$O/lbaprof_$v.txt" 2>&1
  rc=$?; echo "lbaprof $v rc=$rc"; grep LBAPROF "$O/lbaprof_$v.txt" | tail -3; [ $rc -eq 0 ] || exit $rc
done
