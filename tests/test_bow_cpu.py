"""CPU checks of the DBoW2 transform oracle (oracle/bow_oracle.c)."""
import numpy as np

from orbslam2_amd import synth


def _descend_np(voc, f):
    """Independent numpy restatement of TemplatedVocabulary::transform(feature, ...)."""
    par = voc["parent"]
    children = {}
    for i in range(1, len(par)):
        children.setdefault(int(par[i]), []).append(i)
    bits = np.unpackbits(voc["desc"], axis=1)
    fb = np.unpackbits(f)
    node, path = 0, []
    while node in children:
        ch = children[node]
        d = (bits[ch] != fb).sum(1)
        node = ch[int(np.argmin(d))]      # argmin = first minimum
        path.append(node)
    return node, path


def test_oracle_matches_numpy_descent(oracle_mod):
    voc = synth.vocabulary(3, 5, 4)
    leaves = np.nonzero(voc["is_leaf"])[0]
    wid = {int(l): i for i, l in enumerate(leaves)}
    d = synth.bow_features(voc, 1, 300)
    r = oracle_mod.Vocabulary(voc).transform(d, levelsup=2)
    bow = {}
    fv = {}
    for i, f in enumerate(d):
        leaf, path = _descend_np(voc, f)
        w = voc["weight"][leaf]
        if w > 0:
            bow[wid[leaf]] = bow.get(wid[leaf], 0.0) + w
            fv.setdefault(path[4 - 2 - 1], []).append(i)
    words = sorted(bow)
    vals = np.array([bow[w] for w in words])
    vals = vals / np.abs(vals).sum()
    assert r["words"].tolist() == words
    np.testing.assert_allclose(r["values"], vals, rtol=1e-12)
    assert r["fv_nodes"].tolist() == sorted(fv)
    for j, node in enumerate(sorted(fv)):
        assert r["fv_features"][r["fv_start"][j]: r["fv_start"][j + 1]].tolist() == fv[node]


def test_text_roundtrip_oracle(oracle_mod, tmp_path):
    voc = synth.vocabulary(4, 4, 3)
    p = tmp_path / "v.txt"
    p.write_text(synth.vocabulary_text(voc))
    d = synth.bow_features(voc, 2, 200)
    a = oracle_mod.Vocabulary(voc).transform(d)
    b = oracle_mod.Vocabulary(path=str(p)).transform(d)
    for k in a:
        assert a[k].tobytes() == b[k].tobytes()


def test_empty_input(oracle_mod):
    voc = synth.vocabulary(4, 4, 3)
    r = oracle_mod.Vocabulary(voc).transform(np.zeros((0, 32), np.uint8))
    assert len(r["words"]) == 0 and len(r["fv_nodes"]) == 0
