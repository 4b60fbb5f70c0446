"""GPU Frame::ComputeBoW (DBoW2 TemplatedVocabulary::transform, TemplatedVocabulary.h:1125-1286)
vs the CPU oracle, bit-exact: BowVector word ids and double values, FeatureVector nodes and
feature lists. ORBvoc.txt is not in the reference tree, so the vocabularies are synthetic
(synth.vocabulary, same k/L/format); parity against real DBoW2 is unpinned."""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu


def _same(g, r):
    for k in ("words", "values", "fv_nodes", "fv_start", "fv_features"):
        assert g[k].tobytes() == r[k].tobytes(), k


@pytest.fixture(scope="module")
def vocs():
    return {(10, 6): synth.vocabulary(11, 10, 6), (10, 4): synth.vocabulary(12, 10, 4),
            (6, 5): synth.vocabulary(13, 6, 5, stop_frac=0.2)}


@pytest.mark.parametrize("kl,n,levelsup,seed", [((10, 6), 2000, 4, 1), ((10, 6), 4096, 4, 2), ((10, 4), 1000, 2, 3),
                                                ((6, 5), 1500, 4, 4), ((10, 6), 1, 4, 5), ((10, 6), 700, 6, 6),
                                                ((10, 4), 800, 0, 7)])
def test_transform(amd, oracle_mod, vocs, kl, n, levelsup, seed):
    voc = vocs[kl]
    d = synth.bow_features(voc, seed, n)
    g = amd.Vocabulary(voc).transform(d, levelsup)
    r = oracle_mod.Vocabulary(voc).transform(d, levelsup)
    _same(g, r)
    assert len(r["words"]) > 0


@pytest.mark.parametrize("scoring,weighting", [(1, 0), (5, 1), (0, 2), (2, 3), (5, 3)])
def test_scoring_weighting(amd, oracle_mod, vocs, scoring, weighting):
    voc = dict(vocs[(10, 4)], scoring=scoring, weighting=weighting)
    d = synth.bow_features(voc, 9, 1500, noise_bits=8)
    _same(amd.Vocabulary(voc).transform(d), oracle_mod.Vocabulary(voc).transform(d))


def test_text_file_roundtrip(amd, oracle_mod, vocs, tmp_path):
    voc = vocs[(6, 5)]
    path = tmp_path / "voc.txt"
    path.write_text(synth.vocabulary_text(voc))
    d = synth.bow_features(voc, 10, 900)
    g = amd.Vocabulary(path=str(path))
    assert g.info()["n_nodes"] == len(voc["parent"])
    _same(g.transform(d), oracle_mod.Vocabulary(path=str(path)).transform(d))
    _same(g.transform(d), amd.Vocabulary(voc).transform(d))


def test_batched_device(amd, oracle_mod, vocs):
    import torch
    voc = vocs[(10, 6)]
    V, O = amd.Vocabulary(voc), oracle_mod.Vocabulary(voc)
    cap, F = 2048, 12
    descs = [synth.bow_features(voc, 100 + f, 300 + 150 * f) for f in range(F)]
    buf = np.zeros((F, cap, 32), np.uint8)
    cnt = np.zeros(F, np.int32)
    for f, d in enumerate(descs):
        buf[f, : len(d)] = d
        cnt[f] = len(d)
    tb, tc = torch.from_numpy(buf).cuda(), torch.from_numpy(cnt).cuda()
    torch.cuda.synchronize()
    V.transform_batch_device(tb.data_ptr(), tc.data_ptr(), F, cap, cap * 32)
    for f, d in enumerate(descs):
        _same(V.batch_fetch(f, cap), O.transform(d))
