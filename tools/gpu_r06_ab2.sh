#!/bin/bash
# Working tree against a baseline build on one box: the extraction / stereo / RGB-D / matcher /
# headline / new-point parity tests, then alternating C2 (tools/ab_c2.py) and C3 (bench.py's RGB-D
# leg alone) runs:  tools/gpu_r06_ab2.sh <baseline lib.so> [tag]
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
BASE=$1; TAG=${2:-r06_ab2}
timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py tests/test_stereo_gpu.py tests/test_headline_gpu.py \
  tests/test_rgbd_gpu.py tests/test_matcher_gpu.py tests/test_newpts_gpu.py tests/test_host_cpp_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/${TAG}_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$O/${TAG}_tests.log"; [ $rc -eq 0 ] || exit $rc
if [ "${C2:-1}" = 1 ]; then
  timeout -k 10 900 python tools/ab_c2.py "$BASE" orb-slam2-noted_amd/liborbslam2_amd.so ${ROUNDS:-4} > "$O/${TAG}_c2.log" 2>&1
  rc=$?; echo "c2 ab rc=$rc"; grep SUMMARY "$O/${TAG}_c2.log"; [ $rc -eq 0 ] || exit $rc
fi
LEGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --no-e2e"
bash tools/ab_bench.sh "$BASE" orb-slam2-noted_amd/liborbslam2_amd.so ${ROUNDS:-4} $LEGS > "$O/${TAG}_c3.log" 2>&1
rc=$?; echo "c3 ab rc=$rc"
python3 - "$O/${TAG}_c3.log" <<'PY'
import json, sys, collections
v = collections.defaultdict(list)
for line in open(sys.argv[1]):
    tag, js = line.split(' ', 1)
    v[tag].append(json.loads(js)["c3_rgbd_frames_per_s"])
for t, x in v.items(): print("C3", t, round(sum(x) / len(x), 1), x)
PY
exit $rc
