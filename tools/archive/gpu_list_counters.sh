#!/bin/bash
# available PMC counters of this MI355X (TA / TD / TCP / TCC / SQ memory-pipeline names)
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > "$R/gpurun_out/counters.txt" 2>&1
grep -o -E "\b(TA|TD|TCP|SQ_INSTS_VMEM|SQ_INST_CYCLES_VMEM|SQ_WAIT_INST_ANY|SQ_INSTS_FLAT|SQ_LDS|SQC|SQ_IFETCH)[A-Z0-9_]*" "$R/gpurun_out/counters.txt" | sort -u | tr '\n' ' '
