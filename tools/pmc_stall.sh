#!/bin/bash
# Wave-cycle breakdown per extraction kernel (own run, --kernel-trace + --pmc only):
# SQ_WAVE_CYCLES = WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) +
# ACTIVE_INST_ANY (MI355X_MICROARCH.md, SQ counters)
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
TAG="${TAG:-pmc_stall}"   # TAG=lba_stall DRV="lba_prof.py 3": the LocalBA kernels
DRV="${DRV:-prof_extract.py 128 2}"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d "$R/gpurun_out/$TAG" -o run -- python3 "$R/tools/"$DRV > "$R/gpurun_out/$TAG.log" 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && TAG="$TAG" python3 - <<'PY'
import csv, glob, collections, os
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"gpurun_out/{os.environ['TAG']}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1][:28]
        if not k.startswith('__amd'):
            acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in sorted(acc.items()):
    wc = c['SQ_WAVE_CYCLES'] or 1
    print(f"{k:28s} waves {c['SQ_WAVES']:.0f} wave_cyc/wave {wc / max(c['SQ_WAVES'],1):.0f} wait_any {c['SQ_WAIT_ANY']/wc:.2f} "
          f"wait_inst {c['SQ_WAIT_INST_ANY']/wc:.2f} active {c['SQ_ACTIVE_INST_ANY']/wc:.2f} valu {c['SQ_ACTIVE_INST_VALU']/wc:.2f} "
          f"lds {c['SQ_ACTIVE_INST_LDS']/wc:.2f} valu_insts/wave {c['SQ_INSTS_VALU']/max(c['SQ_WAVES'],1):.0f}")
PY
