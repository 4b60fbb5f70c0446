"""bench.py's self-launch, on the CPU: `bench.py --gpus N`
without WORLD_SIZE starts torch.distributed.run with N ranks as a child process and relays rank 0's
JSON line. The ranks here are a stub script (no GPU): the test covers the launcher's contract --
N ranks really start with RANK / WORLD_SIZE set, rank 0's line is relayed, a failing or hanging rank
makes the launcher exit non-zero, and a WORLD_SIZE that differs from --gpus is refused."""
import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

STUB = textwrap.dedent("""
    import json, os, sys, time
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mode = sys.argv[1]
    print(f"rank {rank} chatter", flush=True)
    if mode == "fail" and rank == 1:
        sys.exit(3)
    if mode == "fail_last" and rank == world - 1:
        time.sleep(1)
        sys.exit(5)
    if mode == "hang" and rank == 1:
        time.sleep(600)
    if rank == 0 and mode != "silent":
        print(json.dumps({"metric": "m", "value": 1.0, "n_gpus": world, "argv": sys.argv[1:],
                          "launch": os.environ.get("ORBSLAM_BENCH_LAUNCH")}), flush=True)
""")


@pytest.fixture()
def stub(tmp_path, monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    p = tmp_path / "stub_rank.py"
    p.write_text(STUB)
    return p


def test_self_launch_relays_rank0(stub, capsys):
    rc = bench.self_launch(3, ["ok", "--x"], 120, script=stub)
    out = capsys.readouterr().out.strip().splitlines()
    assert rc == 0
    assert len(out) == 1, out                      # exactly one line on stdout: rank 0's JSON
    doc = json.loads(out[0])
    assert doc["n_gpus"] == 3 and doc["argv"] == ["ok", "--x"] and doc["launch"] == "self"


def test_self_launch_8_ranks(stub, capsys):
    """The driver's N = 8 form: eight ranks start with RANK 0..7, rank 0's line is relayed."""
    rc = bench.self_launch(8, ["ok"], 180, script=stub)
    out = capsys.readouterr()
    assert rc == 0
    assert json.loads(out.out.strip())["n_gpus"] == 8
    assert all(f"rank {r} chatter" in out.err for r in range(8))


def test_self_launch_8_ranks_last_fails(stub, capsys):
    """One failing rank among eight (the last, after rank 0 has printed its line): the launcher exits
    non-zero and relays no line."""
    assert bench.self_launch(8, ["fail_last"], 180, script=stub) != 0
    assert capsys.readouterr().out.strip() == ""


def test_self_launch_rank_failure_is_nonzero(stub, capsys):
    assert bench.self_launch(2, ["fail"], 120, script=stub) != 0
    assert capsys.readouterr().out.strip() == ""


def test_self_launch_no_line_is_nonzero(stub, capsys):
    assert bench.self_launch(2, ["silent"], 120, script=stub) == 1


def test_self_launch_timeout_kills_ranks(stub, capsys):
    assert bench.self_launch(2, ["hang"], 20, script=stub) == 124


def test_world_size_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4"], env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
