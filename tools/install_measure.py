"""Copy a stamped measurement pass (tools/gpu_measure.sh) from gpurun_out/ into profiles/: the two
stamped PMC summaries the bench line reads (box paths in their source lists made repo-relative) and
the rocprofv3 kernel-stats CSVs of the C2 and LocalBA passes, named after the commit they stamp."""
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
O, P = ROOT / "gpurun_out", ROOT / "profiles"


def rel(p):
    s = str(p)
    i = s.find("gpurun_out/")
    return s[i:] if i >= 0 else s


def main():
    commit = None
    for name in ("pmc_traffic.json", "lba_pmc.json"):
        d = json.loads((O / name).read_text())
        commit = d["stamp"]["commit"]
        if isinstance(d.get("source"), list):
            d["source"] = [rel(s) for s in d["source"]]
        (P / name).write_text(json.dumps(d, indent=1) + "\n")
    for src, dst in ((O / "m_trace" / "run_kernel_stats.csv", f"r04_kernel_stats_c2only_{commit}.csv"),
                     (O / "m_lba_stats" / "run_kernel_stats.csv", f"r04_lba_kernel_stats_{commit}.csv")):
        if src.exists():
            shutil.copy(src, P / dst)
            print("copied", dst)
    print("stamped commit", commit)


if __name__ == "__main__":
    sys.exit(main())
