#!/bin/bash
# FETCH_SIZE / WRITE_SIZE against the requested bytes of the round-4 replicas
# (tools/microbench/fetch_calib2.hip; build it on the CPU first). Output:
# gpurun_out/fetch_calib2.json = per kernel: counter bytes / requested bytes.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 "$R/tools/microbench/fetch_calib2" > "$O/fc2_bytes.json" || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d "$O/fc2_$c" -o run --output-format csv -- "$R/tools/microbench/fetch_calib2" > /dev/null 2> "$O/fc2_$c.err"
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$O" <<'PY'
import csv, glob, json, sys
O = sys.argv[1]
nb = json.load(open(f"{O}/fc2_bytes.json"))
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{O}/fc2_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k in nb:
                res.setdefault(k, dict(nb[k]))[c + "_bytes"] = float(r["Counter_Value"]) * 1024
for k, v in res.items():
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        if c + "_bytes" in v:
            v[c + "_per_requested"] = round(v[c + "_bytes"] / v["requested"], 4)
            v[c + "_per_distinct"] = round(v[c + "_bytes"] / v["distinct"], 4)
json.dump(res, open(f"{O}/fetch_calib2.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
