#!/bin/bash
# LocalBA: MFMA PMC pass (per-kernel FP64 MFMA ops / busy cycles) + the Cholesky phase profile
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/lba_pmc" -o run -- python3 "$R/tools/lba_prof.py" 5 > "$R/gpurun_out/lba_pmc.json" 2> "$R/gpurun_out/lba_pmc.err"
rc=$?; cd "$R"; cat gpurun_out/lba_pmc.json; tail -3 gpurun_out/lba_pmc.err; [ $rc -eq 0 ] || exit $rc
ORBSLAM_AMD_LIB="$R/orb-slam2-noted_amd/build/var_lbaprof/liborbslam2_amd.so" timeout -k 10 120 python tools/lba_prof.py 3 > gpurun_out/lba_cholprof.txt 2>&1
rc=$?; grep LBAPROF gpurun_out/lba_cholprof.txt | tail -5; exit $rc
