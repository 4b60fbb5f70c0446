#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / abort / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_if_fatal() {  # $1 = rc, $2 = step; pytest rc 1 (= test failures) is not fatal
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "FATAL rc=$rc in $2" | tee -a $OUT/session.log; exit $rc; fi
}
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
      rc=$?; echo "tests rc=$rc" | tee -a $OUT/session.log; tail -3 $OUT/gpu_tests.log; stop_if_fatal $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" | tee -a $OUT/session.log; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "bench rc=$rc" | tee -a $OUT/session.log; cat $OUT/bench.json; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
      rc=$?; cd "$GRAFT_REPO_ROOT"; echo "prof rc=$rc" | tee -a $OUT/session.log; [ $rc -eq 0 ] || exit $rc
      find $OUT/prof -name "*stats*" ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp
      for ctr in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
        timeout -k 10 600 rocprofv3 --kernel-trace --pmc $ctr -d "$GRAFT_REPO_ROOT/$OUT/pmc_$ctr" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-profile ${PMC_ARGS:---no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency} > /dev/null 2> "$GRAFT_REPO_ROOT/$OUT/pmc_$ctr.err"
        rc=$?; echo "pmc $ctr rc=$rc" | tee -a "$GRAFT_REPO_ROOT/$OUT/session.log"; [ $rc -eq 0 ] || exit $rc
      done
      cd "$GRAFT_REPO_ROOT" ;;
  esac
done
echo "session done" | tee -a $OUT/session.log
