#!/bin/bash
# (Needs tools/exp_resize_tail.patch applied: git apply tools/exp_resize_tail.patch.)
# A/B of the fused coarse-level pyramid launch (ORBX_RESIZE_TAIL = first fused level, 0 = one
# launch per level): extraction / stereo / headline parity with the tail on, then alternating
# C2-only bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for T in ${TAIL_TEST:-4 2}; do
  ORBX_RESIZE_TAIL=$T timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_stereo_gpu.py tests/test_headline_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tail_tests_$T.log 2>&1
  rc=$?; echo "tail=$T tests rc=$rc"; tail -2 gpurun_out/tail_tests_$T.log; [ $rc -eq 0 ] || exit $rc
done
for T in ${TAIL_BENCH:-0 4 3 0 4 3 5}; do
  ORBX_RESIZE_TAIL=$T timeout -k 10 200 python bench.py --no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts > gpurun_out/tail_bench_$T.json 2> gpurun_out/tail_bench_$T.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tail_bench_$T.err; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/tail_bench_$T.json').read().strip().splitlines()[-1]); print('tail=$T', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))" | tee -a gpurun_out/tail_ab.log
done
