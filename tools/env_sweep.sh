#!/bin/bash
# C2-only bench under a sweep of environment settings: env_sweep.sh "A=1 B=2" "A=3" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
k=0
for setting in "$@"; do
  k=$((k+1))
  env $setting timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts ${BENCH_ARGS:-} > gpurun_out/sweep_$k.json 2> gpurun_out/sweep_$k.err || exit $?
  python3 -c "import json,sys;d=json.load(open('gpurun_out/sweep_$k.json'));print('$setting', d['value'], d['kernel_ms_per_step'])"
done
