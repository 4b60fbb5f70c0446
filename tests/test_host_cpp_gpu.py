"""The C++ host layer (orb-slam2-noted_amd/host/orbslam2_amd.hpp: ORBextractor / ORBmatcher /
ComputeStereoMatches / Optimizer::LocalBundleAdjustment with the reference names) driven from
a compiled C++ program, compared with the CPU oracle. This process uses only the /opt/rocm
HIP runtime (no torch)."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "orb-slam2-noted_amd" / "build" / "host_api_test"
KP = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
               ("octave", "<i4"), ("class_id", "<i4")])


def _read(path, dtypes):
    buf = path.read_bytes()
    out, off = [], 0
    for dt in dtypes:
        n = int(np.frombuffer(buf, np.int64, 1, off)[0])
        off += 8
        a = np.frombuffer(buf, dt, n, off).copy()
        off += n * np.dtype(dt).itemsize
        out.append(a)
    return out


def _run(*args):
    if not EXE.exists():
        import __graft_entry__
        __graft_entry__.build()
    r = subprocess.run([str(EXE), *map(str, args)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr


def test_cpp_extract(tmp_path, oracle_mod):
    img = synth.textured_image(480, 640, 77)
    (tmp_path / "img.u8").write_bytes(img.tobytes())
    _run("extract", tmp_path / "img.u8", 640, 480, 1000, tmp_path / "out.bin")
    kps, desc, sf = _read(tmp_path / "out.bin", [KP, np.uint8, np.float32])
    rk, rd = oracle_mod.Extractor(1000).extract(img)
    assert kps.tobytes() == rk.tobytes()
    assert np.array_equal(desc.reshape(-1, 32), rd)
    np.testing.assert_array_equal(sf, oracle_mod.Extractor(1000).scale_factors)


def test_cpp_stereo(tmp_path, oracle_mod):
    L, R = synth.stereo_pair(376, 1241, 5)
    (tmp_path / "l.u8").write_bytes(L.tobytes())
    (tmp_path / "r.u8").write_bytes(R.tobytes())
    mb = float(np.float32(386.1448) / np.float32(718.856))
    _run("stereo", tmp_path / "l.u8", tmp_path / "r.u8", 1241, 376, 2000, repr(386.1448), repr(mb), tmp_path / "o.bin")
    u, d = _read(tmp_path / "o.bin", [np.float32, np.float32])
    exL, exR = oracle_mod.Extractor(2000), oracle_mod.Extractor(2000)
    kL, dL = exL.extract(L)
    kR, dR = exR.extract(R)
    ru, rd = oracle_mod.stereo_matches(exL, exR, kL, dL, kR, dR, np.float32(386.1448), np.float32(mb))
    assert u.tobytes() == ru.tobytes() and d.tobytes() == rd.tobytes()


def _lba_blob(prob):
    np_, nq, ne = len(prob["pose_id"]), len(prob["point_id"]), len(prob["edge_point"])
    parts = [np.array([np_, nq, ne], np.int32).tobytes(), prob["pose_id"].astype(np.int32).tobytes(),
             prob["pose_fixed"].astype(np.uint8).tobytes(), b"\0" * ((4 - np_ % 4) % 4),
             prob["pose_Tcw"].astype(np.float32).tobytes(), prob["pose_cam"].astype(np.float32).tobytes(),
             prob["point_id"].astype(np.int32).tobytes(), prob["point_Xw"].astype(np.float32).tobytes(),
             prob["edge_point"].astype(np.int32).tobytes(), prob["edge_pose"].astype(np.int32).tobytes(),
             prob["edge_obs"].astype(np.float32).tobytes(), prob["edge_inv_sigma2"].astype(np.float32).tobytes()]
    return b"".join(parts)


def test_cpp_concurrent_frame_threads_and_localba(tmp_path, oracle_mod):
    """Frame.cc:144-153 runs the left / right ORBextractor on two std::threads while the
    LocalMapping thread runs LocalBundleAdjustment (LocalMapping.cc:116-118). 12 rounds of L || R
    extraction + ComputeStereoMatches with LocalBA running back to back on a third thread: every
    round bit-exact with the serial run and with the oracle, every LocalBA within 1e-4 of the
    oracle with the same erase set."""
    L, R = synth.stereo_pair(376, 1241, 6)
    (tmp_path / "l.u8").write_bytes(L.tobytes())
    (tmp_path / "r.u8").write_bytes(R.tobytes())
    prob = synth.localba_problem(seed=9, n_kf=10, n_points=600)
    (tmp_path / "p.bin").write_bytes(_lba_blob(prob))
    mb = float(np.float32(386.1448) / np.float32(718.856))
    rounds = 12
    _run("concurrent", tmp_path / "l.u8", tmp_path / "r.u8", 1241, 376, 2000, repr(386.1448), repr(mb),
         tmp_path / "p.bin", rounds, tmp_path / "o.bin")
    buf = (tmp_path / "o.bin").read_bytes()
    hdr, ms = _read_prefix(buf, [np.int32, np.float64])
    mism, nr, nlba = (int(v) for v in hdr)
    assert nr == rounds and mism == 0, f"{mism} of {rounds} concurrent rounds differ from the serial run"
    assert nlba >= 2
    # serial run vs oracle (extraction + stereo), once
    exL, exR = oracle_mod.Extractor(2000), oracle_mod.Extractor(2000)
    kL, dL = exL.extract(L)
    kR, dR = exR.extract(R)
    _run("stereo", tmp_path / "l.u8", tmp_path / "r.u8", 1241, 376, 2000, repr(386.1448), repr(mb), tmp_path / "s.bin")
    u, d = _read(tmp_path / "s.bin", [np.float32, np.float32])
    ru, rd = oracle_mod.stereo_matches(exL, exR, kL, dL, kR, dR, np.float32(386.1448), np.float32(mb))
    assert u.tobytes() == ru.tobytes() and d.tobytes() == rd.tobytes()
    ref = oracle_mod.lba_solve(prob)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    arrs = _read(tmp_path / "o.bin", [np.int32, np.float64] + [np.float32, np.float32, np.uint8] * nlba)[2:]
    for i in range(nlba):
        T, X, er = arrs[3 * i: 3 * i + 3]
        assert rel(T.reshape(-1, 16).astype(np.float64), ref["pose_Tcw"]) < 1e-4
        assert rel(X.reshape(-1, 3).astype(np.float64), ref["point_Xw"]) < 1e-4
        assert np.array_equal(er, ref["edge_erase"])


def _read_prefix(buf, dtypes):
    out, off = [], 0
    for dt in dtypes:
        n = int(np.frombuffer(buf, np.int64, 1, off)[0])
        off += 8
        out.append(np.frombuffer(buf, dt, n, off).copy())
        off += n * np.dtype(dt).itemsize
    return out


def test_cpp_localba(tmp_path, oracle_mod):
    prob = synth.localba_problem(seed=9, n_kf=10, n_points=600)
    np_, nq, ne = len(prob["pose_id"]), len(prob["point_id"]), len(prob["edge_point"])
    parts = [np.array([np_, nq, ne], np.int32).tobytes(), prob["pose_id"].astype(np.int32).tobytes(),
             prob["pose_fixed"].astype(np.uint8).tobytes(), b"\0" * ((4 - np_ % 4) % 4),
             prob["pose_Tcw"].astype(np.float32).tobytes(), prob["pose_cam"].astype(np.float32).tobytes(),
             prob["point_id"].astype(np.int32).tobytes(), prob["point_Xw"].astype(np.float32).tobytes(),
             prob["edge_point"].astype(np.int32).tobytes(), prob["edge_pose"].astype(np.int32).tobytes(),
             prob["edge_obs"].astype(np.float32).tobytes(), prob["edge_inv_sigma2"].astype(np.float32).tobytes()]
    (tmp_path / "p.bin").write_bytes(b"".join(parts))
    _run("lba", tmp_path / "p.bin", tmp_path / "o.bin")
    T, X, er = _read(tmp_path / "o.bin", [np.float32, np.float32, np.uint8])
    ref = oracle_mod.lba_solve(prob)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    assert rel(T.reshape(-1, 16).astype(np.float64), ref["pose_Tcw"]) < 1e-4
    assert rel(X.reshape(-1, 3).astype(np.float64), ref["point_Xw"]) < 1e-4
    assert np.array_equal(er, ref["edge_erase"])


def test_cpp_pose_optimization(tmp_path, oracle_mod):
    p = synth.pose_problem(21, n=500)
    n = len(p["Xw"])
    blob = (np.array([n], np.int32).tobytes() + np.asarray(p["Tcw"], np.float32).tobytes() +
            np.array(p["cam"], np.float32).tobytes() + p["Xw"].astype(np.float32).tobytes() +
            p["obs"].astype(np.float32).tobytes() + p["inv_sigma2"].astype(np.float32).tobytes())
    (tmp_path / "e.bin").write_bytes(blob)
    _run("pose", tmp_path / "e.bin", tmp_path / "o.bin")
    T, out, nin = _read(tmp_path / "o.bin", [np.float32, np.uint8, np.int32])
    ref = oracle_mod.pose_optimization(p)
    assert int(nin[0]) == ref["n_inliers"] and np.array_equal(out, ref["outlier"])
    assert np.abs(T.reshape(4, 4).astype(np.float64) - ref["Tcw"]).max() < 1e-4


def test_cpp_bow_text_vocabulary(tmp_path, oracle_mod):
    voc = synth.vocabulary(31, 8, 4)
    (tmp_path / "voc.txt").write_text(synth.vocabulary_text(voc))
    d = synth.bow_features(voc, 5, 1200)
    (tmp_path / "d.u8").write_bytes(d.tobytes())
    _run("bow", tmp_path / "voc.txt", tmp_path / "d.u8", len(d), 4, tmp_path / "o.bin")
    words, vals, nodes, start, feats = _read(tmp_path / "o.bin", [np.uint32, np.float64, np.uint32, np.int32, np.int32])
    ref = oracle_mod.Vocabulary(voc).transform(d, 4)
    assert words.tobytes() == ref["words"].tobytes() and vals.tobytes() == ref["values"].tobytes()
    assert nodes.tobytes() == ref["fv_nodes"].tobytes() and start.tobytes() == ref["fv_start"].tobytes()
    assert feats.tobytes() == ref["fv_features"].tobytes()


def test_host_local_mapping_triangulate(oracle_mod, tmp_path):
    """LocalMapping::TriangulateMatches (host C++ over orbn_triangulate) vs the oracle."""
    prob = synth.newpoints_problem(seed=41)
    blob = [np.array([len(prob["kf1"]["keys"]), len(prob["kf2"]["keys"]), len(prob["pairs"])], np.int32).tobytes(),
            np.float32(prob["ratio_factor"]).tobytes()]
    for k in (prob["kf1"], prob["kf2"]):
        blob += [np.ascontiguousarray(k["keys"]).view(KP).tobytes(), np.ascontiguousarray(k["keys_un"]).view(KP).tobytes(),
                 np.asarray(k["u_right"], np.float32).tobytes(), np.asarray(k["depth"], np.float32).tobytes()]
        hdr = np.concatenate([np.asarray(k["Tcw"], np.float32).reshape(-1), np.asarray(k["Ow"], np.float32),
                              np.array([k[f] for f in ("fx", "fy", "cx", "cy", "invfx", "invfy", "mb", "mbf")], np.float32)])
        blob += [hdr.astype(np.float32).tobytes(), np.int32(k["nlevels"]).tobytes()]
        for f in ("scale_factors", "level_sigma2"):
            a = np.zeros(16, np.float32)
            a[: k["nlevels"]] = k[f]
            blob.append(a.tobytes())
    blob.append(np.ascontiguousarray(prob["pairs"], np.int32).tobytes())
    (tmp_path / "p.bin").write_bytes(b"".join(blob))
    subprocess.run([str(EXE), "newpts", str(tmp_path / "p.bin"), str(tmp_path / "o.bin")], check=True, timeout=120)
    nnew, x3d, ok = _read(tmp_path / "o.bin", [np.int32, np.float32, np.uint8])
    rn, rx, rok = oracle_mod.triangulate(prob)
    assert int(nnew[0]) == rn
    np.testing.assert_array_equal(ok, rok)
    assert x3d.tobytes() == rx.reshape(-1).tobytes()
