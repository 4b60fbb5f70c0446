"""CPU checks of the BoW-matcher oracle restatements (oracle/track_oracle.c)."""
import numpy as np

from orbslam2_amd import synth


def _bruteforce_bow(p, nnratio=0.7):
    """Pure-Python restatement of SearchByBoW without the rotation check (small case)."""
    A, B = p["A"], p["B"]
    nodesB = {int(n): j for j, n in enumerate(B["fv_nodes"])}
    bits = lambda d: np.unpackbits(d)
    out = [-1] * len(B["keys_un"])
    nm = 0
    for a, node in enumerate(A["fv_nodes"]):
        if int(node) not in nodesB:
            continue
        j = nodesB[int(node)]
        fb = B["fv_features"][B["fv_start"][j]:B["fv_start"][j + 1]]
        for ia in A["fv_features"][A["fv_start"][a]:A["fv_start"][a + 1]]:
            if A["mp"][ia] < 0 or A["mp_bad"][ia]:
                continue
            b1 = b2 = 256
            bi = -1
            for ib in fb:
                if out[ib] >= 0:
                    continue
                d = int((bits(A["desc"][ia]) != bits(B["desc"][ib])).sum())
                if d < b1:
                    b2, b1, bi = b1, d, ib
                elif d < b2:
                    b2 = d
            if b1 <= 50 and np.float32(b1) < np.float32(nnratio) * np.float32(b2):
                out[bi] = int(A["mp"][ia])
                nm += 1
    return nm, np.array(out, np.int32)


def test_search_by_bow_oracle_vs_python(oracle_mod):
    p = synth.bow_match_problem(21, n=300, n_points=250)
    nm, m = oracle_mod.search_by_bow(p, 0.7, check_ori=False)
    nm2, m2 = _bruteforce_bow(p, 0.7)
    assert nm == nm2 and np.array_equal(m, m2)


def test_triangulation_pairs_sorted_and_unique(oracle_mod):
    p = synth.bow_match_problem(22, n=1500, n_points=1200)
    r = oracle_mod.search_for_triangulation(p)
    assert len(r) > 0
    assert np.all(np.diff(r[:, 0]) > 0)                  # idx1 ascending, unique
    assert len(np.unique(r[:, 1])) == len(r)             # vbMatched2: each idx2 once
    assert (p["A"]["mp"][r[:, 0]] < 0).all() and (p["B"]["mp"][r[:, 1]] < 0).all()
