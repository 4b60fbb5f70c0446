#!/bin/bash
# fast_blur_kernel with / without XCD-aware block runs (build/var_fbxcd64): isolated wave-cycle
# breakdown (tools/pmc_stall.sh) and vector-memory pipeline load (tools/pmc_mem.sh), one engine
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
for v in base fbxcd64; do
  if [ $v = base ]; then unset ORBSLAM_AMD_LIB; else export ORBSLAM_AMD_LIB="$R/orb-slam2-noted_amd/build/var_$v/liborbslam2_amd.so"; fi
  TAG=stall_$v bash tools/pmc_stall.sh > "$O/fbxcd_stall_$v.txt" 2>&1; rc=$?; echo "stall $v rc=$rc"; grep -E "fast_blur|resize" "$O/fbxcd_stall_$v.txt"; [ $rc -eq 0 ] || exit $rc
  bash tools/pmc_mem.sh > "$O/fbxcd_mem_$v.txt" 2>&1; rc=$?; echo "mem $v rc=$rc"; grep -E "fast_blur|resize" "$O/fbxcd_mem_$v.txt"; [ $rc -eq 0 ] || exit $rc
done
