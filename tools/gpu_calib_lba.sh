#!/bin/bash
# One GPU session: fetch-size calibration microbenches + request-size PMC passes over them and over
# the C2 leg (tools/pmc_reqsize.sh), then an A/B of a LocalBA variant library against the product:
#   tools/gpu_calib_lba.sh <variant lib.so>
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
V=$1
O=$R/gpurun_out; mkdir -p "$O"
MB=$R/tools/microbench
LEGS="--no-cpu-baseline --no-profile --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency"
timeout -k 10 120 "$MB/fetch_calib" > "$O/fc1_bytes.json" &&
timeout -k 10 120 "$MB/fetch_calib2" > "$O/fc2_bytes.json" &&
bash "$R/tools/pmc_reqsize.sh" fc1 "$MB/fetch_calib" &&
bash "$R/tools/pmc_reqsize.sh" fc2 "$MB/fetch_calib2" &&
bash "$R/tools/pmc_reqsize.sh" c2 python3 "$R/bench.py" --steps 3 --warmup 1 --no-lba $LEGS &&
cd "$R" &&
ORBSLAM_AMD_LIB=$(realpath "$V") timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py -x -q --timeout 120 \
  --timeout-method thread > "$O/variant_lba_tests.log" 2>&1 && echo "variant lba tests ok" &&
bash "$R/tools/ab_bench.sh" "$R/orb-slam2-noted_amd/liborbslam2_amd.so" "$V" 3 --no-c2 --steps 1 --warmup 1 \
  --lba-steps 30 $LEGS > "$O/ab_lba.log" 2>&1 && echo "ab done"
