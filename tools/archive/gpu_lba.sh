#!/bin/bash
# LocalBA measurement session: FP64 MFMA peak, counter names, C4 wall time, kernel trace + stats
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_all.txt 2>&1; grep -i -E "mfma|f64|fp64" gpurun_out/counters_all.txt | head -80 > gpurun_out/counters_mfma.txt
timeout -k 10 60 tools/microbench/mfma_f64_peak > gpurun_out/mfma_f64_peak.json || exit $?
cat gpurun_out/mfma_f64_peak.json
timeout -k 10 120 python tools/lba_prof.py 30 > gpurun_out/lba_wall.json || exit $?
cat gpurun_out/lba_wall.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/lba_prof" -o run -- python3 "$R/tools/lba_prof.py" 30 > "$R/gpurun_out/lba_prof.json" 2> "$R/gpurun_out/lba_prof.err"
rc=$?; cd "$R"; cat gpurun_out/lba_prof.json; exit $rc
