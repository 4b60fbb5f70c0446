#!/bin/bash
# Pipeline shape sweep (tools/pipeline_exp.py) + single-engine kernel stats of the C2 leg
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/pipeline_exp.py ${CASES:-256,1,plain 384,1,plain 384,2,alt 384,3,alt 384,2,free 384,3,free 512,4,free} > gpurun_out/pipe.txt 2>&1
rc=$?; cat gpurun_out/pipe.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof1" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-profile --engines 1 --batch 256 --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-e2e > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1.err"
rc=$?; cd "$R"; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof1/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
