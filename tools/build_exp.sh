#!/bin/bash
# Build an experiment library from the working tree's sources with one file replaced, into
# orb-slam2-noted_amd/build/exp_<name>/ (same flags as the product build), for same-box A/B runs:
#   tools/build_exp.sh <name> <csrc file to replace> <replacement file>
set -eu
NAME=$1; F=$2; REPL=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/orb-slam2-noted_amd/build/exp_$NAME
TMP=$(mktemp -d)
mkdir -p "$OUT" "$TMP/orb-slam2-noted_amd" "$TMP/build"
cp -r "$ROOT/orb-slam2-noted_amd/csrc" "$TMP/orb-slam2-noted_amd/"; cp -r "$ROOT/include" "$TMP/"
cp "$REPL" "$TMP/orb-slam2-noted_amd/csrc/$F"
echo "#define ORBX_SRC_HASH \"exp_$NAME\"" > "$TMP/build/build_id.h"
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
