#!/bin/bash
# Drop-in latency: stereo_latency (threads + serial) and a kernel trace of it with the L / R overlap summary
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
python -c "
import numpy as np, sys
sys.path.insert(0,'orb-slam2-noted_amd/python')
from orbslam2_amd import synth
with open('/tmp/pairs.u8','wb') as f:
    for t in range(8):
        L,R=synth.stereo_pair(376,1241,2+t); f.write(L.tobytes()); f.write(R.tobytes())
"
EXE="$R/orb-slam2-noted_amd/build/stereo_latency"
for m in threads serial; do
  timeout -k 10 120 "$EXE" /tmp/pairs.u8 8 1241 376 2000 386.1448 0.5371789 16 ${FRAMES:-512} $m || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/lat_trace" -o run -- "$EXE" /tmp/pairs.u8 8 1241 376 2000 386.1448 0.5371789 4 32 threads > "$R/gpurun_out/lat_trace.json" 2> "$R/gpurun_out/lat_trace.err"
rc=$?; cd "$R"; cat gpurun_out/lat_trace.json; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/lat_trace -name "*kernel_trace.csv" | head -1)
python tools/latency_overlap.py "$f" > gpurun_out/lat_overlap.txt; tail -1 gpurun_out/lat_overlap.txt
