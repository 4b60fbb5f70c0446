#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on this MI355X for the access widths the extraction kernels
# use (tools/microbench/fetch_calib.hip; build it on the CPU first). Output:
# gpurun_out/fetch_calib.json = per kernel: counter bytes / distinct bytes touched.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 "$R/tools/microbench/fetch_calib" > "$O/fc_bytes.json" || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d "$O/fc_$c" -o run --output-format csv -- "$R/tools/microbench/fetch_calib" > /dev/null 2> "$O/fc_$c.err"
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$O" <<'PY'
import csv, glob, json, sys
O = sys.argv[1]
nbytes = json.load(open(f"{O}/fc_bytes.json"))
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{O}/fc_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k in nbytes:
                res.setdefault(k, {"bytes": nbytes[k]})[c + "_bytes"] = float(r["Counter_Value"]) * 1024
for k, v in res.items():
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        if c + "_bytes" in v:
            v[c + "_ratio"] = round(v[c + "_bytes"] / v["bytes"], 4)
json.dump(res, open(f"{O}/fetch_calib.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
