#!/bin/bash
# Isolated per-kernel durations and wave counters of the extraction kernels (one BatchExtractor,
# 128 pairs, tools/prof_extract.py) for each setting in KPROF_ENVS (space-separated VAR=v,VAR=v
# lists; "base" = no extra variables). Own run per counter pass.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out/kprof"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for e in ${KPROF_ENVS:-base}; do
  n=$(echo "$e" | tr ',=' '__')
  envs=(); [ "$e" = base ] || IFS=',' read -ra envs <<< "$e"
  env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/t_$n" -o run -- python3 "$R/tools/prof_extract.py" 128 3 > /dev/null 2>&1 || exit $?
  env "${envs[@]}" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$O/p_$n" -o run -- python3 "$R/tools/prof_extract.py" 128 2 > /dev/null 2>&1 || exit $?
  python3 - "$O/t_$n" "$O/p_$n" "$e" <<'PY'
import csv, glob, sys, collections
t = {}
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        t[r['Name'].split('(')[0].replace('void ', '').split('::')[-1]] = float(r['AverageNs']) / 1e3
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[2] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1]
        acc[k][r['Counter_Name']] += float(r['Counter_Value']); disp[k].add(r['Dispatch_Id'])
print('==', sys.argv[3])
for k in sorted(t):
    if k.startswith('__amd'): continue
    c = acc.get(k, {}); w = max(c.get('SQ_WAVES', 0), 1); n = max(len(disp.get(k, ())), 1)
    print(f"{k:28s} avg_us {t[k]:9.1f}  valu/launch {c.get('SQ_INSTS_VALU',0)/n/1e6:7.2f}M valu/wave {c.get('SQ_INSTS_VALU',0)/w:6.0f} "
          f"salu/wave {c.get('SQ_INSTS_SALU',0)/w:5.0f} lds/wave {c.get('SQ_INSTS_LDS',0)/w:5.0f} parked {c.get('SQ_WAIT_ANY',0)/max(c.get('SQ_WAVE_CYCLES',1),1):.2f} cyc/wave {c.get('SQ_WAVE_CYCLES',0)/w:6.0f}")
PY
done
