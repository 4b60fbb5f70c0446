#!/bin/bash
# Vector-memory pipeline load of the extraction kernels (tools/prof_extract.py, one engine, 128
# pairs): TA / TD busy cycles against the kernel's duration, VMEM instructions per wave. One
# counter pass per block, each in its own run.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out/pmc_mem"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/t" -o run -- python3 "$R/tools/prof_extract.py" 128 2 > /dev/null 2>&1 || exit $?
i=0
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/p$i" -o run -- python3 "$R/tools/prof_extract.py" 128 2 > /dev/null 2>&1 || exit $?
  i=$((i+1))
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
dur = {}
for r in csv.DictReader(open(glob.glob(O + '/t/**/*kernel_stats.csv', recursive=True)[0])):
    dur[r['Name'].split('(')[0].replace('void ', '').split('::')[-1]] = float(r['AverageNs']) * 1e-9
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in glob.glob(O + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1]
        acc[k][r['Counter_Name']] += float(r['Counter_Value']); disp[k][r['Counter_Name']].add(r['Dispatch_Id'])
CLK, CUS = 2.4e9, 256
for k in sorted(dur):
    if k.startswith('__amd') or k not in acc: continue
    c = acc[k]; n = lambda name: max(len(disp[k][name]), 1)
    cyc = dur[k] * CLK * CUS
    w = c['SQ_WAVES'] or 1
    print(f"{k:28s} us {dur[k]*1e6:7.1f} TA_busy {c['TA_TA_BUSY_sum']/n('TA_TA_BUSY_sum')/cyc:5.2f} TA_stall_TC {c['TA_ADDR_STALLED_BY_TC_CYCLES_sum']/n('TA_ADDR_STALLED_BY_TC_CYCLES_sum')/cyc:5.2f} "
          f"TD_busy {c['TD_TD_BUSY_sum']/n('TD_TD_BUSY_sum')/cyc:5.2f} TD_TC_stall {c['TD_TC_STALL_sum']/n('TD_TC_STALL_sum')/cyc:5.2f} vmem_rd/wave {c['SQ_INSTS_VMEM_RD']/w:6.1f} vmem_wr/wave {c['SQ_INSTS_VMEM_WR']/w:5.1f} lds/wave {c['SQ_INSTS_LDS']/w:5.1f}")
PY
