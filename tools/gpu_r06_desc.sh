#!/bin/bash
# Round-6 describe2 load-order fix: exhaustive sincosf equivalence, the extraction / stereo / RGB-D /
# headline / new-point parity tests, then the same-box C2 A/B against a baseline build:
#   tools/gpu_r06_desc.sh <baseline lib.so> [tag]
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
BASE=$1; TAG=${2:-r06_desc}
timeout -k 10 120 tools/microbench/sincosf_equiv > "$O/${TAG}_sincosf.json" 2>&1
rc=$?; echo "sincosf rc=$rc $(cat "$O/${TAG}_sincosf.json")"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py tests/test_stereo_gpu.py tests/test_headline_gpu.py \
  tests/test_rgbd_gpu.py tests/test_newpts_gpu.py tests/test_host_cpp_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$O/${TAG}_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$O/${TAG}_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/ab_c2.py "$BASE" orb-slam2-noted_amd/liborbslam2_amd.so ${ROUNDS:-4} > "$O/${TAG}_ab.log" 2>&1
rc=$?; echo "ab rc=$rc"; grep SUMMARY "$O/${TAG}_ab.log"; exit $rc
