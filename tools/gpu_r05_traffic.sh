#!/bin/bash
# Traffic (request-size PMC passes, C2 leg only, 3 + 1 steps) of the working-tree library and of the
# variants named in $@, then same-box C2 A/Bs of the working tree against each variant.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
C2ONLY="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize --no-profile"
for tag in prod "$@"; do
  LIB="$R/orb-slam2-noted_amd/liborbslam2_amd.so"; [ "$tag" = prod ] || LIB="$R/orb-slam2-noted_amd/build/var_$tag/liborbslam2_amd.so"
  ORBSLAM_AMD_LIB="$LIB" bash tools/pmc_reqsize.sh "t_$tag" python3 "$R/bench.py" --steps 3 --warmup 1 $C2ONLY || exit $?
  python3 tools/reqsize_summary.py "$O" "t_$tag" > "$O/r05_traffic_$tag.json" 2>&1 || exit $?
  python3 - "$O/r05_traffic_$tag.json" "$tag" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
tot = 0
for k, e in sorted(d.items()):
    if not isinstance(e, dict) or "traffic_bytes" not in e: continue
    tot += e["traffic_bytes"] * e["launches"]
    print(sys.argv[2], k, e["launches"], round(e["read_bytes"] / 1e6, 1), "MB rd", round(e["write_bytes"] / 1e6, 1), "MB wr")
print(sys.argv[2], "TOTAL over the run (4 steps)", round(tot / 1e9, 3), "GB; per step", round(tot / 4e9, 3), "GB")
PY
done
for tag in "$@"; do
  timeout -k 10 900 python tools/ab_c2.py "$R/orb-slam2-noted_amd/liborbslam2_amd.so" "$R/orb-slam2-noted_amd/build/var_$tag/liborbslam2_amd.so" 3 > "$O/r05_ab_c2_$tag.log" 2>&1
  rc=$?; echo "ab $tag rc=$rc"; grep SUMMARY "$O/r05_ab_c2_$tag.log"; [ $rc -eq 0 ] || exit $rc
done
