#!/bin/bash
# resize_pyramid_kernel: extraction parity tests (every resize / blur mode, sizes, flush), the headline
# and C3 shape tests, smoke; then a same-box A/B of the fused pyramid against the per-level launches
# (the knobs variant with ORBX_RZ_FUSED=0 / 1) and its traffic.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_extract_gpu.py tests/test_headline_gpu.py tests/test_stereo_gpu.py tests/test_rgbd_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/r05_rz_tests.log" 2>&1
rc=$?; tail -3 "$O/r05_rz_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
K="$R/orb-slam2-noted_amd/build/var_knobs/liborbslam2_amd.so"
timeout -k 10 900 env ORBX_RZ_FUSED=0 python tools/ab_c2.py "$K" "$R/orb-slam2-noted_amd/liborbslam2_amd.so" 3 > "$O/r05_ab_rz_fused.log" 2>&1
rc=$?; echo "ab rc=$rc"; grep SUMMARY "$O/r05_ab_rz_fused.log"; [ $rc -eq 0 ] || exit $rc
C2ONLY="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize --no-profile"
bash tools/pmc_reqsize.sh t_rzf python3 "$R/bench.py" --steps 3 --warmup 1 $C2ONLY || exit $?
python3 tools/reqsize_summary.py "$O" t_rzf > "$O/r05_traffic_rzf.json" 2>&1 || exit $?
python3 - "$O/r05_traffic_rzf.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); tot = 0
for k, e in sorted(d.items()):
    if not isinstance(e, dict) or "traffic_bytes" not in e: continue
    tot += e["traffic_bytes"] * e["launches"]
    print(k, e["launches"], round(e["read_bytes"] / 1e6, 1), "MB rd", round(e["write_bytes"] / 1e6, 1), "MB wr")
print("per step", round(tot / 4e9, 3), "GB")
PY
