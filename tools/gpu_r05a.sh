#!/bin/bash
# Round-5 session A: the full GPU parity suite, smoke and the default bench line of the working tree,
# then same-box A/Bs of this round's kernel changes against variant builds of the same sources
# (make variant: describe2 without the clipped patch / IC loads, lba_chol_tiled with the
# barrier-per-block back substitution) and the LocalBA Cholesky's phase split (LBA_PROFILE).
# Every GPU step has its own limit; the first failure ends the session.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
V="$R/orb-slam2-noted_amd/build"
STEPS="${STEPS:-tests smoke bench abdesc ablba lbaprof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/r05_gpu_tests.log" 2>&1
      rc=$?; echo "tests rc=$rc"; tail -4 "$O/r05_gpu_tests.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/r05_smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -1 "$O/r05_smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py > "$O/r05_bench.json" 2> "$O/r05_bench.err"
      rc=$?; echo "bench rc=$rc"; head -c 1500 "$O/r05_bench.json"; echo; [ $rc -eq 0 ] || exit $rc ;;
    abdesc)
      timeout -k 10 900 python tools/ab_c2.py "$R/orb-slam2-noted_amd/liborbslam2_amd.so" "$V/var_noclip/liborbslam2_amd.so" 4 > "$O/r05_ab_desc_clip.log" 2>&1
      rc=$?; echo "abdesc rc=$rc"; grep SUMMARY "$O/r05_ab_desc_clip.log"; [ $rc -eq 0 ] || exit $rc ;;
    ablba)
      LEGS="--no-c2 --no-cpu-baseline --no-profile --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --steps 1 --warmup 1 --lba-steps 40"
      timeout -k 10 600 bash tools/ab_bench.sh "$V/var_solve16/liborbslam2_amd.so" "$R/orb-slam2-noted_amd/liborbslam2_amd.so" 4 $LEGS > "$O/r05_ab_lba_solve.log" 2>&1
      rc=$?; echo "ablba rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python3 - "$O/r05_ab_lba_solve.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag, js = line.split(' ', 1)
    l = json.loads(js)["localba"]
    print(tag, l["ms_per_call"], l["gpu_ms_per_call"], l["host_ms_per_call"], l["kernel_ms_per_call"].get("lba_chol_tiled"))
PY
      ;;
    lbaprof)
      ORBSLAM_AMD_LIB="$V/var_lbaprof/liborbslam2_amd.so" timeout -k 10 120 python3 tools/lba_prof.py 3 > "$O/r05_lbaprof.txt" 2>&1
      rc=$?; echo "lbaprof rc=$rc"; grep LBAPROF "$O/r05_lbaprof.txt" | tail -3; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo "session done"
