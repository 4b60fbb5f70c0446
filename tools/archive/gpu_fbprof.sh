#!/bin/bash
# fast_blur phase profile (clock64 per phase, sampled blocks) on the C2 batch shape
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
ORBSLAM_AMD_LIB="$R/orb-slam2-noted_amd/build/var_fbprof/liborbslam2_amd.so" timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-e2e --batch 12 --engines 1 > gpurun_out/fbprof.txt 2>&1
rc=$?; grep -c FBPROF gpurun_out/fbprof.txt; exit $rc
