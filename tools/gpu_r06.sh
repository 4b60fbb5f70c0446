#!/bin/bash
# Round-6 GPU session of the working tree: the full GPU parity suite, smoke and the default bench
# line (STEPS selects; every step has its own limit and the first failure ends the session).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
TAG="${TAG:-r06}"
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-} > "$O/${TAG}_gpu_tests.log" 2>&1
      rc=$?; echo "tests rc=$rc"; tail -4 "$O/${TAG}_gpu_tests.log"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -1 "$O/${TAG}_smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err"
      rc=$?; echo "bench rc=$rc"; head -c 400 "$O/${TAG}_bench.json"; echo; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo "session done"
