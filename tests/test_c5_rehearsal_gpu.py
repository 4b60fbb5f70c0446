"""C5 rehearsal: bench.py's multi-rank path at world size 2 on the one GPU of
the box, launched by bench.py itself: `bench.py --gpus 2` without WORLD_SIZE starts
torch.distributed.run with two ranks as a child process and relays rank 0's line,
over gloo (ORBSLAM_DIST_BACKEND=gloo: ranks share the card, RCCL needs one GPU per rank). Each rank runs
its own 512-frame C2 stream (SURVEY §8d C5 seeds: rank r's frame t = seed 10 + r + 8 t), receives the LocalBA map from rank 0
by broadcast, and checks with --check-parity its whole last 384-pair batch bit-exact and its
LocalBA on the broadcast map within 1e-4 (same LM iterations, same erase set) against the oracle.
The multi-rank timing is a rehearsal, not a measurement (two ranks share one GPU)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_c5_two_ranks_parity():
    env = dict(os.environ, ORBSLAM_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    env = {k: v for k, v in env.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--launch-timeout", "220",
           "--steps", "3", "--warmup", "1", "--check-parity", "--no-cpu-baseline", "--no-latency",
           "--no-e2e", "--no-rgbd", "--no-track", "--no-pose", "--no-bow", "--no-bowmatch", "--no-newpts",
           "--no-isolated", "--no-alt-resize", "--lba-steps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    log = ROOT / "gpurun_out"
    if log.is_dir():
        (log / "c5_rehearsal.log").write_text(r.stdout + "\n--- stderr ---\n" + r.stderr)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "ms_per_step", "parity_check")}))
    assert line["n_gpus"] == 2 and "C5" in line["config"]["streams"]
    cfg = line["config"]
    assert cfg["world_size"] == 2 and cfg["dist_backend"] == "gloo", cfg
    assert cfg["launch"].startswith("bench.py self-launch"), cfg
    assert [d["rank"] for d in cfg["rank_devices"]] == [0, 1], cfg
    c2 = line["parity_check"]["c2"]
    assert [p["rank"] for p in c2] == [0, 1]
    for r, p in enumerate(c2):   # rank r's stream: frame t from seed 10 + r + 8 t
        assert p["left_seed_first_pair"] == 10 + r + 8 * p["first_frame"], p
        assert p["pairs_checked"] == 384 and p["pairs_bit_exact"] == 384 and p["distinct_pairs"] == 384, p
    lba = line["localba"]["parity_check"]
    assert len(lba) == 2 and lba[0]["map_bytes"] == lba[1]["map_bytes"] > 0
    for p in lba:
        assert p["within_1e-4"] and p["same_lm_iterations"] and p["same_erase_set"], p


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_single_rank():
    """The RCCL path itself on the box's one GPU (RCCL never executed): torch.distributed.run
    with one rank, backend nccl (= RCCL), process group bound to the rank's device, and with
    ORBSLAM_DIST_FORCE=1 every collective of the multi-rank bench (shared parameters, the LocalBA map
    broadcast, barriers, the max-over-ranks timing, the parity gather) runs through RCCL at world size 1.
    xGMI between GPUs stays unexercised here: the driver's 8-GPU node runs that."""
    env = dict(os.environ, ORBSLAM_DIST_FORCE="1", PYTHONUNBUFFERED="1")
    env.pop("ORBSLAM_DIST_BACKEND", None)
    env = {k: v for k, v in env.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--check-parity", "--no-cpu-baseline", "--no-latency",
           "--no-e2e", "--no-rgbd", "--no-track", "--no-pose", "--no-bow", "--no-bowmatch", "--no-newpts",
           "--no-isolated", "--no-alt-resize", "--lba-steps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    log = ROOT / "gpurun_out"
    if log.is_dir():
        (log / "rccl_single_rank.log").write_text(r.stdout + "\n--- stderr ---\n" + r.stderr)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "ms_per_step")}))
    cfg = line["config"]
    assert cfg["world_size"] == 1 and cfg["dist_backend"] == "rccl (torch nccl)", cfg
    assert cfg["launch"] == "external torch.distributed.run", cfg
    assert line["localba"]["map_source"] == "rank 0, RCCL broadcast"
    c2 = line["parity_check"]["c2"]
    assert len(c2) == 1 and c2[0]["pairs_checked"] == 384 and c2[0]["pairs_bit_exact"] == 384, c2
    (lba,) = line["localba"]["parity_check"]
    assert lba["map_bytes"] > 0 and lba["within_1e-4"] and lba["same_lm_iterations"] and lba["same_erase_set"], lba
