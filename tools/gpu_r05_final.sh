#!/bin/bash
# Round-5 final measurement session of the working tree (GIT_HEAD=<commit> in the environment):
# the full GPU parity suite, smoke, the default bench line, the stamped C2 counters and LocalBA PMC of
# tools/gpu_measure.sh (kernel-trace stats, FETCH / WRITE / VALU, request sizes, MFMA), and the C3
# leg's rocprofv3 summary. Every step has its own limit; the first failure ends the session.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/r05_final_gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$O/r05_final_gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/r05_final_smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$O/r05_final_smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$O/r05_final_bench.json" 2> "$O/r05_final_bench.err"
rc=$?; echo "bench rc=$rc"; head -c 600 "$O/r05_final_bench.json"; echo; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_measure.sh; rc=$?; echo "measure rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_c3_prof.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
echo "final session done"
