#!/bin/bash
# LocalBA: parity tests, wall, Cholesky variants, kernel stats + MFMA PMC pass of the default build
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
VARIANTS="${VARIANTS-lbaprof n1 prio n1prio}" bash "$R/tools/gpu_lba_iter.sh" || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/lba_stats" "$R/gpurun_out/lba_pmc"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/lba_stats" -o run -- python3 "$R/tools/lba_prof.py" 30 > "$R/gpurun_out/lba_stats.json" 2> "$R/gpurun_out/lba_stats.err" || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/lba_pmc" -o run -- python3 "$R/tools/lba_prof.py" 5 > "$R/gpurun_out/lba_pmc.json" 2> "$R/gpurun_out/lba_pmc.err" || exit $?
cd "$R"
python tools/lba_pmc_summary.py gpurun_out/lba_pmc/run_counter_collection.csv gpurun_out/lba_stats/run_kernel_stats.csv gpurun_out/r02_lba_pmc.json > /dev/null
cat gpurun_out/lba_stats.json
