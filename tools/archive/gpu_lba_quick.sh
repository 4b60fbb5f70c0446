#!/bin/bash
# LocalBA iteration: parity tests, wall per call with the host phases, per-kernel rocprof stats
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py tests/test_host_cpp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/lba_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lba_tests.log; [ $rc -eq 0 ] || exit $rc
ORBX_LBA_HOSTPROF=1 timeout -k 10 120 python tools/lba_prof.py 20 > gpurun_out/lba_host.log 2>&1 || exit $?
tail -4 gpurun_out/lba_host.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/lq" -o run -- python3 "$R/tools/lba_prof.py" 5 > /dev/null 2>&1 || exit $?
python3 - "$R/gpurun_out/lq" <<'PY'
import csv, glob, sys
for r in csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0])):
    print(f"{r['Name'].split('(')[0].split('::')[-1][:28]:28s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:7.2f}")
PY
