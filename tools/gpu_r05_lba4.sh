#!/bin/bash
# LocalBA: tests + A/B against build/var_$1 (tools/gpu_r05_lba.sh), then the phase split of the
# LBA_PROFILE builds named in the remaining arguments (tools/gpu_lbaprof.sh)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
V=$1; shift
bash tools/gpu_r05_lba.sh "$V"; rc=$?; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_lbaprof.sh "$@"
