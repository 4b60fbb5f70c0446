#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C3 leg (4 engines, 40 batches) for the working-tree library
# and a variant ($1), plus one engine alone (--rgbd-engines 1) for each: per-kernel durations.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"
ARGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --no-e2e"
cd /tmp && export TMPDIR=/tmp
for tag in prod $1; do
  LIB="$R/orb-slam2-noted_amd/liborbslam2_amd.so"; [ "$tag" = prod ] || LIB="$R/orb-slam2-noted_amd/build/var_$tag/liborbslam2_amd.so"
  for eng in 4 1; do
    ORBSLAM_AMD_LIB="$LIB" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c3p_${tag}_e$eng" -o run -- python3 "$R/bench.py" $ARGS --rgbd-steps 40 --rgbd-engines $eng > "$O/c3p_${tag}_e$eng.json" 2> "$O/c3p_${tag}_e$eng.err"
    rc=$?; echo "c3 prof $tag e$eng rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
