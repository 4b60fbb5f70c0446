#!/bin/bash
# Stamped measurement pass of the current library on one MI355X (run through gpurun, with
# GIT_HEAD=<commit> in the environment):
#   1. C2-only rocprofv3 --kernel-trace --stats (the bench line's kernel durations; no isolated
#      or alternate-resize launches, so the CSV average is the line's avg_launch_ms)
#   2. C2-only PMC passes FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU, one counter per pass, and the
#      three request-size passes of tools/pmc_reqsize.sh (exact read / write bytes per kernel)
#      -> gpurun_out/pmc_traffic.json (stamped: tools/stamp.py)
#   3. LocalBA MFMA PMC pass + its kernel stats -> gpurun_out/lba_pmc.json (stamped)
# Copy gpurun_out/{pmc_traffic,lba_pmc}.json and the stats CSVs into profiles/ afterwards.
# Every GPU step has its own time limit and the script stops at the first failure.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
O="$R/gpurun_out"
C2ONLY="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize"
STEPS="${MEASURE:-trace pmc lba}"
cd /tmp && export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/m_trace" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 $C2ONLY ${BENCH_ARGS:-} > "$O/m_trace_bench.json" 2> "$O/m_trace.err"
      rc=$?; echo "trace rc=$rc"; cat "$O/m_trace_bench.json"; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
        timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d "$O/m_pmc_$ctr" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-profile $C2ONLY ${BENCH_ARGS:-} > /dev/null 2> "$O/m_pmc_$ctr.err"
        rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
      bash "$R/tools/pmc_reqsize.sh" m python3 "$R/bench.py" --steps 3 --warmup 1 --no-profile $C2ONLY ${BENCH_ARGS:-}
      rc=$?; echo "pmc reqsize rc=$rc"; [ $rc -eq 0 ] || exit $rc
      REQSIZE_DIR="$O" REQSIZE_TAG=m STEPS_PROFILED=4 python3 "$R/tools/pmc_summary.py" "$O/m_pmc_FETCH_SIZE" "$O/m_pmc_WRITE_SIZE" 128 "$O/pmc_traffic.json" "$O/m_pmc_SQ_INSTS_VALU" > /dev/null
      rc=$?; echo "pmc summary rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    lba)
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/m_lba_stats" -o run -- python3 "$R/tools/lba_prof.py" 5 > "$O/m_lba_stats.txt" 2>&1
      rc=$?; echo "lba stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/m_lba_pmc" -o run -- python3 "$R/tools/lba_prof.py" 5 > "$O/m_lba_pmc.txt" 2>&1
      rc=$?; echo "lba pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python3 "$R/tools/lba_pmc_summary.py" "$(find "$O/m_lba_pmc" -name '*counter_collection.csv' | head -1)" "$(find "$O/m_lba_stats" -name '*kernel_stats.csv' | head -1)" "$O/lba_pmc.json" > /dev/null
      rc=$?; echo "lba summary rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo "measure done"
