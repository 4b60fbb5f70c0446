#!/bin/bash
# e2e (host-batch) leg against the number of HIP hardware queues and pipeline engines: the
# 3 engine streams + H2D + D2H streams exceed GPU_MAX_HW_QUEUES=4 and share queues.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency"
for q in ${QUEUES:-4 8}; do
  for a in ${ENGINES:-3 2}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py $BASE --e2e-engines $a > gpurun_out/e2eq.json 2> gpurun_out/e2eq.err || { tail -3 gpurun_out/e2eq.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/e2eq.json'))
print('queues $q engines $a', 'value', d['value'], 'e2e', d['value_e2e'], d['e2e']['ms_per_step'])" | tee -a gpurun_out/e2eq.txt
  done
done
