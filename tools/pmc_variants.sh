#!/bin/bash
# SQ_INSTS_VALU / SQ_INSTS_LDS / SQ_WAVES of tools/prof_extract.py per library variant
# (build/var_<name>/liborbslam2_amd.so; "base" = the in-tree library), one rocprofv3 pass each
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
    lib="$R/orb-slam2-noted_amd/liborbslam2_amd.so"
    [ "$v" = base ] || lib="$R/orb-slam2-noted_amd/build/var_$v/liborbslam2_amd.so"
    ORBSLAM_AMD_LIB="$lib" timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU --output-format csv -d "$R/gpurun_out/pmcv_$v" -o run -- python3 "$R/tools/prof_extract.py" 128 2 > "$R/gpurun_out/pmcv_$v.log" 2>&1
    rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$R"
python3 - <<'PY'
import csv, glob, collections, os
for d in sorted(glob.glob('gpurun_out/pmcv_*')):
    if not os.path.isdir(d): continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1]
            if not k.startswith('__amd'):
                acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, c in sorted(acc.items()):
        print(d, k, {n: round(sum(v) / len(v)) for n, v in c.items()})
PY
