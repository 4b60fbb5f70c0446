#!/bin/bash
# Same-box A/B of one bench.py leg over two library builds, alternating (ORBSLAM_AMD_LIB):
#   tools/ab_bench.sh <lib_a.so> <lib_b.so> <rounds> <bench.py args...>
# prints one JSON line per run, tagged with the library's directory.
set -u
A=$1; B=$2; N=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "$N"); do
  for L in "$A" "$B"; do
    out=$(ORBSLAM_AMD_LIB=$(realpath "$L") timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1) || exit $?
    echo "$(basename "$(dirname "$L")") $out"
  done
done
