#!/bin/bash
# Build the product library of git revision $1 into orb-slam2-noted_amd/build/ab_<rev>/ (same flags
# as the Makefile's product build) for same-box A/B runs against the working tree:
#   ORBSLAM_AMD_LIB=orb-slam2-noted_amd/build/ab_<rev>/liborbslam2_amd.so python tools/ab_c2.py
set -eu
REV=${1:?revision}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/orb-slam2-noted_amd/build/ab_$REV
TMP=$(mktemp -d)
mkdir -p "$OUT" "$TMP/csrc" "$TMP/include" "$TMP/build"
git -C "$ROOT" archive "$REV" orb-slam2-noted_amd/csrc include | tar -x -C "$TMP"
echo "#define ORBX_SRC_HASH \"ab_$REV\"" > "$TMP/build/build_id.h"
cd "$TMP/orb-slam2-noted_amd"
objs=()
for f in csrc/*.hip; do
  o=$TMP/build/$(basename "$f" .hip).o
  extra=""
  [ "$(basename "$f")" = orb_extract.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
    -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-function -I"$TMP/include" -Icsrc -I"$TMP/build" \
    $extra -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/liborbslam2_amd.so" "${objs[@]}"
rm -rf "$TMP"
echo "$OUT/liborbslam2_amd.so"
