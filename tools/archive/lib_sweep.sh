#!/bin/bash
# C2-only bench line per library variant (build/var_<name>/liborbslam2_amd.so) and bench arg set
# VARIANTS="th16 th24" ARGSETS="--engines 3|--engines 1 --batch 256"
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency"
IFS='|' read -ra SETS <<< "${ARGSETS:---engines 3}"
IFS='|' read -ra ENVS <<< "${ENVSETS:-NONE=0}"
for ev in "${ENVS[@]}"; do
export "$ev"
for v in $VARIANTS; do
  lib="$R/orb-slam2-noted_amd/build/var_$v/liborbslam2_amd.so"; [ "$v" = base ] && lib="$R/orb-slam2-noted_amd/liborbslam2_amd.so"
  for a in "${SETS[@]}"; do
    ORBSLAM_AMD_LIB="$lib" timeout -k 10 200 python bench.py $BASE $a > gpurun_out/sweep.json 2> gpurun_out/sweep.err
    rc=$?; [ $rc -eq 0 ] || { echo "$v [$a] rc=$rc"; tail -3 gpurun_out/sweep.err; exit $rc; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sweep.json')); r=d['roofline']
print('$ev', '$v', '[$a]', d['value'], 'fb_ms', r['avg_launch_ms'], {k: v for k, v in d['kernel_ms_per_step'].items()})" | tee -a gpurun_out/sweep.txt
  done
done
unset "${ev%%=*}"
done
