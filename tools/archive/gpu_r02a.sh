#!/bin/bash
# round-2 check: host-mode / concurrency tests, C2 + e2e + latency bench, kernel trace of the latency driver
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stereo_gpu.py tests/test_matcher_gpu.py tests/test_host_cpp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err
rc=$?; cat gpurun_out/r02a_bench.json; tail -3 gpurun_out/r02a_bench.err; [ $rc -eq 0 ] || exit $rc
python -c "
import numpy as np, sys
sys.path.insert(0,'orb-slam2-noted_amd/python')
from orbslam2_amd import synth
with open('/tmp/pairs.u8','wb') as f:
    for t in range(8):
        L,R=synth.stereo_pair(376,1241,2+t); f.write(L.tobytes()); f.write(R.tobytes())
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/lat_trace" -o run -- "$R/orb-slam2-noted_amd/build/stereo_latency" /tmp/pairs.u8 8 1241 376 2000 386.1448 0.5371789 4 32 threads > "$R/gpurun_out/lat_trace.json" 2> "$R/gpurun_out/lat_trace.err"
rc=$?; cd "$R"; cat gpurun_out/lat_trace.json; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/lat_trace -name "*kernel_trace.csv" | head -1)
python tools/latency_overlap.py "$f" > gpurun_out/lat_overlap.txt; tail -1 gpurun_out/lat_overlap.txt
