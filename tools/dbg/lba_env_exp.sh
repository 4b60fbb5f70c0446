# C4 LocalBA wall time per call under HIP runtime settings (one process each)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
for v in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "" ; do
  echo "== [$v]"; env $v timeout -k 10 120 python3 tools/lba_prof.py 40 2>/dev/null | tail -1 || exit $?
done
