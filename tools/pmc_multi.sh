#!/bin/bash
# Counter passes over tools/prof_extract.py: one rocprofv3 run per pass (--kernel-trace + --pmc
# only), output under gpurun_out/pmc_<pass>/. Usage: pmc_multi.sh [batch]
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
B="${1:-128}"
run() {
    local name="$1"; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc_$name" -o run -- \
        python3 "$R/tools/prof_extract.py" "$B" 2 > "$R/gpurun_out/pmc_$name.log" 2>&1
    local rc=$?
    echo "pass $name rc=$rc"
    return $rc
}
run occ SQ_WAVES SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES &&
run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TA_TOTAL_WAVEFRONTS_sum &&
run spi SPI_RA_WAVE_SIMD_FULL_CSN SPI_RA_VGPR_SIMD_FULL_CSN SPI_RA_LDS_CU_FULL_CSN SPI_RA_TGLIM_CU_FULL_CSN SPI_RA_RES_STALL_CSN SPI_CSN_BUSY SPI_RA_REQ_NO_ALLOC_CSN SPI_RA_BAR_CU_FULL_CSN
