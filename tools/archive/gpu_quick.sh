#!/bin/bash
# Quick GPU check: extraction + stereo parity tests, then a C2-only bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TESTS="${TESTS:-tests/test_extract_gpu.py tests/test_stereo_gpu.py}"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_FLAGS:---no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts} ${BENCH_ARGS:-} > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
rc=$?; cat gpurun_out/quick_bench.json; tail -3 gpurun_out/quick_bench.err; exit $rc
