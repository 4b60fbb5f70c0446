#!/bin/bash
# Round-6 final session of the committed tree (GIT_HEAD=<commit>): GPU suite, smoke, bench line,
# stamped C2 / LocalBA counters (tools/gpu_measure.sh) and the C3 leg's rocprofv3 summary.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
TAG="r06_${GIT_HEAD:?commit}" bash tools/gpu_r06.sh || exit $?
bash tools/gpu_measure.sh || exit $?
bash tools/gpu_c3_prof.sh || exit $?
echo "final done"
