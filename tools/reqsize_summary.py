#!/usr/bin/env python3
"""Per-kernel L2 -> fabric traffic from the request-size counters of tools/pmc_reqsize.sh:
read bytes = 32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B, write bytes = 64 WRREQ_64B + 32 (WRREQ -
WRREQ_64B), averaged per dispatch; FETCH_SIZE-equivalent (64 x RDREQ) beside them.
  reqsize_summary.py <gpurun_out dir> <tag> [bytes.json of known per-kernel byte counts]"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def short(name):
    return name.split("(")[0].replace("void ", "").split("::")[-1]


def load(d: Path):
    acc = defaultdict(lambda: defaultdict(list))
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def summarize(out_dir: Path, tag: str, known=None):
    c = defaultdict(dict)
    for p in ("rd32_64", "rd128_all", "wr"):
        for k, cs in load(out_dir / f"rq_{tag}_{p}").items():
            for name, vals in cs.items():
                c[k][name] = (sum(vals) / len(vals), len(vals))
    res = {}
    for k, cs in c.items():
        g = lambda n: cs.get(n, (0.0, 0))[0]
        rd = 32 * g("TCC_EA0_RDREQ_32B") + 64 * g("TCC_EA0_RDREQ_64B") + 128 * g("TCC_EA0_RDREQ_128B")
        wr = 64 * g("TCC_EA0_WRREQ_64B") + 32 * (g("TCC_EA0_WRREQ") - g("TCC_EA0_WRREQ_64B"))
        e = {"launches": max(v[1] for v in cs.values()), "read_bytes": int(rd), "write_bytes": int(wr),
             "traffic_bytes": int(rd + wr), "fetch_size_equiv_bytes": int(64 * g("TCC_EA0_RDREQ")),
             "rdreq": {"32B": g("TCC_EA0_RDREQ_32B"), "64B": g("TCC_EA0_RDREQ_64B"), "128B": g("TCC_EA0_RDREQ_128B"),
                       "all": g("TCC_EA0_RDREQ")}}
        if e["fetch_size_equiv_bytes"]:
            e["read_factor_vs_fetch_size"] = round(rd / e["fetch_size_equiv_bytes"], 4)
        if known and k in known:
            kb = known[k]
            e["known"] = kb
            for kk in ("requested", "distinct"):
                if isinstance(kb, dict) and kb.get(kk):
                    e[f"read_per_{kk}"] = round(rd / kb[kk], 4)
                    e[f"write_per_{kk}"] = round(wr / kb[kk], 4)
            if isinstance(kb, (int, float)) and kb:
                e["read_per_known"] = round(rd / kb, 4)
                e["write_per_known"] = round(wr / kb, 4)
        res[k] = e
    return res


if __name__ == "__main__":
    d, tag = Path(sys.argv[1]), sys.argv[2]
    known = {}
    for f in sys.argv[3:]:
        known.update(json.load(open(f)))
    r = summarize(d, tag, known)
    print(json.dumps(r, indent=1))
