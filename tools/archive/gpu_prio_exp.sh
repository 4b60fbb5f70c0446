cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
L=orb-slam2-noted_amd
timeout -k 10 500 python tools/skip_exp.py base=$L/liborbslam2_amd.so fb1=$L/build/var_fb1/liborbslam2_amd.so fb2rz=$L/build/var_fb2rz/liborbslam2_amd.so base2=$L/liborbslam2_amd.so > gpurun_out/prio.log 2>&1
rc=$?; cat gpurun_out/prio.log; exit $rc
