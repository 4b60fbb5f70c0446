#!/bin/bash
# Round-6 A/B of lever (a), the GaussianBlur inside the descriptor kernel (describe3_kernel, no blurred
# pyramid): parity of the variant build on every extraction / stereo / headline / RGB-D GPU test
# (both blur modes), then the same-box C2 A/B against the baseline variant (tools/ab_c2.py). First, the
# product's LocalBA large-window leg (bench.py localba_windows).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
V=orb-slam2-noted_amd/build/var_descblur/liborbslam2_amd.so
B=orb-slam2-noted_amd/build/var_base/liborbslam2_amd.so
timeout -k 10 300 python bench.py --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency \
  --no-cpu-baseline --steps 5 > "$O/r06_lba_windows.json" 2> "$O/r06_lba_windows.err"
rc=$?; echo "lba windows rc=$rc"; [ $rc -eq 0 ] || exit $rc
ORBSLAM_AMD_LIB=$(realpath $V) timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py tests/test_stereo_gpu.py \
  tests/test_headline_gpu.py tests/test_rgbd_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$O/r06_descblur_tests.log" 2>&1
rc=$?; echo "variant tests rc=$rc"; tail -4 "$O/r06_descblur_tests.log"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/ab_c2.py $B $V 4 > "$O/r06_ab_descblur.log" 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 "$O/r06_ab_descblur.log"; [ $rc -eq 0 ] || exit $rc
echo done
