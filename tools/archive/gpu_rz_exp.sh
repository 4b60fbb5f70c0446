#!/bin/bash
# Resize chain stream of the stereo pipeline (ORBX_PIPE_RZ: 0 engine stream, 1 own stream, 2 own
# high-priority stream), same box, one experiment build read through the environment; then the
# product build's parity tests and a C2 kernel trace of the product default:
#   tools/gpu_rz_exp.sh <variant lib.so>
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
V=$(realpath "$1")
cd "$R"
timeout -k 10 120 python3 -c "import torch; print(\"priority range (least, greatest):\", torch.cuda.Stream.priority_range())" | tee -a "$OUT/rz_exp.log"
C2="--no-cpu-baseline --no-lba --no-rgbd --no-track --no-pose --no-bow --no-bowmatch --no-newpts --no-e2e --no-latency --no-isolated --no-alt-resize --steps 40"
for rep in 1 2; do
  for m in 0 2 3 4 1; do
    line=$(ORBSLAM_AMD_LIB=$V ORBX_PIPE_RZ=$m timeout -k 10 180 python3 bench.py $C2 2>/dev/null | tail -1) || exit $?
    echo "rz=$m $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_ms"], json.dumps(d.get("kernel_ms_per_step")))' "$line")" | tee -a "$OUT/rz_exp.log"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py tests/test_stereo_gpu.py tests/test_headline_gpu.py tests/test_host_cpp_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/rz_tests.log" 2>&1
rc=$?; tail -2 "$OUT/rz_tests.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rz_trace" -o run -- python3 "$R/bench.py" $C2 --steps 10 --warmup 2 --no-profile > "$OUT/rz_trace_bench.json" 2> "$OUT/rz_trace.err"
echo "trace rc=$?"
