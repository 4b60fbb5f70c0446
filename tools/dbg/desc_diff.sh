cd ${GRAFT_REPO_ROOT:-/root/repo}
for v in ${DESC_VS:-82 42 0}; do ORBX_DESC_V=$v timeout -k 10 120 python tools/dbg/desc_diff.py || exit $?; done
