"""bench.py publishes committed PMC counters (profiles/pmc_traffic.json, profiles/lba_pmc.json) only
for the library they were measured on: the summary's stamp.src_hash (tools/src_hash.py at profiling
time) must equal the loaded library's orbx_build_id(), and the stamped configuration must match the
run. CPU only: the stamp check itself and the committed summaries' shape."""
import json
from pathlib import Path

import pytest

import bench

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture
def profiles(tmp_path, monkeypatch):
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "ROOT", tmp_path)

    def write(name, stamp, kernels):
        (tmp_path / "profiles" / name).write_text(json.dumps({"stamp": stamp, "kernels": kernels}))
    return write


def test_matching_stamp_publishes_counters(profiles):
    profiles("p.json", {"src_hash": "abc", "commit": "c0ffee", "batch": 128, "resize_mode": 0},
             {"orbamd::fast_blur_kernel(orbamd::ExtractGeom, ...)": {"valu_insts_per_launch": 7}})
    kern, note = bench.load_pmc_doc("p.json", "abc", batch=128, resize_mode=0)
    assert kern is not None and kern["fast_blur_kernel"]["valu_insts_per_launch"] == 7
    assert "abc" in note and "c0ffee" in note


def test_other_sources_withhold_counters(profiles):
    profiles("p.json", {"src_hash": "abc", "commit": "c0ffee", "batch": 128}, {"k": {}})
    kern, note = bench.load_pmc_doc("p.json", "def", batch=128)
    assert kern is None and "not reported" in note


def test_other_configuration_withholds_counters(profiles):
    profiles("p.json", {"src_hash": "abc", "commit": "c0ffee", "batch": 128, "resize_mode": 0}, {"k": {}})
    kern, note = bench.load_pmc_doc("p.json", "abc", batch=256, resize_mode=0)
    assert kern is None and "batch" in note
    kern, note = bench.load_pmc_doc("p.json", "abc", batch=128, resize_mode=1)
    assert kern is None and "resize_mode" in note


def test_missing_or_unstamped_summary(profiles):
    kern, note = bench.load_pmc_doc("absent.json", "abc")
    assert kern is None and "absent" in note
    profiles("old.json", None, {"k": {}})
    kern, note = bench.load_pmc_doc("old.json", "abc")
    assert kern is None


@pytest.mark.parametrize("fname", ["pmc_traffic.json", "lba_pmc.json"])
def test_committed_summaries_are_stamped(fname):
    doc = json.loads((ROOT / "profiles" / fname).read_text())
    st = doc["stamp"]
    assert len(st["src_hash"]) == 16 and int(st["src_hash"], 16) >= 0
    assert st["commit"] and st["commit"] != "unknown"
    assert doc["kernels"]


def _counter_csv(d: Path, rows):
    d.mkdir(parents=True)
    lines = ["Kernel_Name,Counter_Name,Counter_Value"] + [f'"{k}",{c},{v}' for k, c, v in rows]
    (d / "run_counter_collection.csv").write_text("\n".join(lines) + "\n")


def test_reqsize_summary_bytes(tmp_path):
    """Exact traffic from the request-size passes: 32/64/128-B read requests and 64-B / other write
    requests, averaged per dispatch (tools/reqsize_summary.py)."""
    import sys
    sys.path.insert(0, str(ROOT / "tools"))
    from reqsize_summary import summarize
    k = "void orbamd::fast_blur_kernel<false>(orbamd::ExtractGeom, ...)"
    _counter_csv(tmp_path / "rq_t_rd32_64", [(k, "TCC_EA0_RDREQ_32B", 10), (k, "TCC_EA0_RDREQ_64B", 100),
                                               (k, "TCC_EA0_RDREQ_32B", 30), (k, "TCC_EA0_RDREQ_64B", 300)])
    _counter_csv(tmp_path / "rq_t_rd128_all", [(k, "TCC_EA0_RDREQ_128B", 1000), (k, "TCC_EA0_RDREQ", 1220),
                                                (k, "TCC_EA0_RDREQ_128B", 1000), (k, "TCC_EA0_RDREQ", 1220)])
    _counter_csv(tmp_path / "rq_t_wr", [(k, "TCC_EA0_WRREQ", 500), (k, "TCC_EA0_WRREQ_64B", 400)])
    e = summarize(tmp_path, "t")["fast_blur_kernel<false>"]
    assert e["launches"] == 2
    assert e["read_bytes"] == 32 * 20 + 64 * 200 + 128 * 1000
    assert e["write_bytes"] == 64 * 400 + 32 * 100
    assert e["traffic_bytes"] == e["read_bytes"] + e["write_bytes"]
    assert e["fetch_size_equiv_bytes"] == 64 * 1220


def test_step_traffic_published(profiles):
    """A summary carrying step_traffic_bytes (every dispatch of a step) hands it to the bench line."""
    (Path(bench.ROOT) / "profiles" / "p.json").write_text(json.dumps(
        {"stamp": {"src_hash": "abc", "commit": "c0ffee", "batch": 128}, "step_traffic_bytes": 12345,
         "kernels": {"k": {"read_bytes_per_launch": 1, "write_bytes_per_launch": 2}}}))
    kern, _ = bench.load_pmc_doc("p.json", "abc", batch=128)
    assert kern["__step_traffic__"] == 12345 and kern["k"]["write_bytes_per_launch"] == 2
