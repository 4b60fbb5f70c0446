#!/bin/bash
# Same-box A/B of the LocalBA leg: product library against each variant build given, alternating.
#   tools/gpu_ab_lba_vars.sh <variant lib.so>...
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
PROD="$R/orb-slam2-noted_amd/liborbslam2_amd.so"
LEGS="--no-c2 --no-cpu-baseline --no-profile --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --steps 1 --warmup 1 --lba-steps 40"
for V in "$@"; do
  bash tools/ab_bench.sh "$PROD" "$V" 3 $LEGS >> "$OUT/ab_lba_vars.log" 2>&1 || exit $?
done
python3 - "$OUT/ab_lba_vars.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag, js = line.split(' ', 1)
    l = json.loads(js)["localba"]
    print(tag, l["ms_per_call"], l["kernel_ms_per_call"].get("lba_chol_tiled"), l["lm_trials"])
PY
