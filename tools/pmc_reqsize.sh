#!/bin/bash
# L2 -> fabric request counts by size, for exact traffic bytes (FETCH_SIZE tallies every read
# request at 64 B: half of a 128-B streaming request, a 32-B request at double). Three passes,
# two TCC counters each, over the same command:
#   tools/pmc_reqsize.sh <tag> <command...>     -> gpurun_out/rq_<tag>_{rd32_64,rd128_all,wr}/
set -u
TAG=$1; shift
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {   # $1 = pass name, $2.. = counters
  local p=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d "$O/rq_${TAG}_$p" -o run --output-format csv -- "${CMD[@]}" > /dev/null 2> "$O/rq_${TAG}_$p.err"
  local rc=$?; echo "pmc $TAG $p rc=$rc"; return $rc
}
CMD=("$@")
run rd32_64 TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B && run rd128_all TCC_EA0_RDREQ_128B TCC_EA0_RDREQ && \
  run wr TCC_EA0_WRREQ TCC_EA0_WRREQ_64B
