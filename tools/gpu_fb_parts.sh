#!/bin/bash
# fast_blur_kernel VALU / duration by part: FB_SKIP_* builds (tools/prof_extract.py, one engine)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out/fbparts"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for nv in base=orb-slam2-noted_amd/liborbslam2_amd.so ${FB_VARS:-}; do
  n=${nv%%=*}; lib=${nv#*=}
  ORBSLAM_AMD_LIB="$R/$lib" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d "$O/$n" -o run -- python3 "$R/tools/prof_extract.py" 128 2 > /dev/null 2>&1 || exit $?
  python3 - "$O/$n" "$n" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set); dur = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].split('::')[-1].split('<')[0]
        acc[k][r['Counter_Name']] += float(r['Counter_Value']); disp[k].add(r['Dispatch_Id'])
k = 'fast_blur_kernel'; c = acc[k]; n = len(disp[k]); w = c['SQ_WAVES']
print(f"{sys.argv[2]:8s} fast_blur valu/launch {c['SQ_INSTS_VALU']/n/1e6:7.2f}M valu/wave {c['SQ_INSTS_VALU']/w:6.1f} lds/wave {c['SQ_INSTS_LDS']/w:5.1f} salu/wave {c['SQ_INSTS_SALU']/w:5.1f}")
PY
done
