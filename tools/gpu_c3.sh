#!/bin/bash
# C3 (RGB-D) leg alone: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes (separate runs),
# and which HIP / HSA runtimes one bench process maps (torch's bundled vs /opt/rocm's).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
ARGS="--no-c2 --no-lba --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-latency --no-cpu-baseline --no-profile --rgbd-steps 10"
cd "$R"
timeout -k 10 120 python3 - > "$OUT/runtime_maps.txt" 2>&1 <<'PY'
import sys; sys.path.insert(0, "orb-slam2-noted_amd/python")
import torch; torch.cuda.init(); x = torch.zeros(4, device="cuda")
import orbslam2_amd as amd; amd.lib(); print("devices", amd.device_count())
seen = set()
for line in open("/proc/self/maps"):
    p = line.split()[-1]
    if any(k in p for k in ("amdhip64", "hsa-runtime", "rccl", "orbslam2")) and p not in seen:
        seen.add(p); print(p)
PY
echo "maps rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3prof" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/c3_bench.json" 2> "$OUT/c3_prof.err"
rc=$?; echo "c3 prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT/c3pmc_$ctr" -o run -- python3 "$R/bench.py" $ARGS --rgbd-steps 2 > /dev/null 2> "$OUT/c3pmc_$ctr.err"
  rc=$?; echo "c3 pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
