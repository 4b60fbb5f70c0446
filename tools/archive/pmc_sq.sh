#!/bin/bash
# SQ counter pass over tools/prof_extract.py (own run, --kernel-trace + --pmc only)
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmc_sq" -o run -- python3 "$R/tools/prof_extract.py" 128 2 > "$R/gpurun_out/pmc_sq.log" 2>&1
echo "rc=$?"
