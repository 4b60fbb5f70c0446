#!/bin/bash
# C2 leg of a variant build under several fast_blur LDS reservations (ORBX_FB_LDS_PAD bytes per
# workgroup: 0 = 8 workgroups per CU, 1400 = 7, 4300 = 6, 8000 = 5), alternating, 3 rounds:
#   tools/archive/gpu_fb_pad.sh <variant lib.so> [pads...]  (needs tools/archive/exp_fb_lds_pad.patch applied)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
LIB=$(realpath "$1"); shift
PADS="${*:-0 1400 4300 8000}"
LEGS="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize --steps 40 --warmup 3"
for r in 1 2 3; do
  for p in $PADS; do
    out=$(ORBX_FB_LDS_PAD=$p ORBSLAM_AMD_LIB=$LIB timeout -k 10 300 python bench.py $LEGS 2>/dev/null | tail -1) || exit $?
    echo "$out" | python3 -c "
import json,sys; b=json.loads(sys.stdin.read()); k=b['kernel_ms_per_step']
print('pad $p', b['value'], b['ms_per_step'], k.get('fast_blur_kernel'), k.get('resize_level_kernel'), k.get('describe2_kernel'), flush=True)"
  done
done
