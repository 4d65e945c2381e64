"""Load a torch-path RONI golden (tests/golden/gen_roni_softmax_goldens.py):
the inputs, regenerated from the case seed and checked against the stored
SHA-256, and the reference's scores / correct counts / last-batch indices."""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def names():
    return sorted(json.load(open(os.path.join(HERE, "roni_softmax_cases.json"))))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()


def load(name):
    import gen_roni_softmax_goldens as G  # make_case only; never touches the reference
    p = G.CASES[name]
    g = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    X, y, ww, D = G.make_case(**p)
    for a, key in ((X, "X_sha256"), (ww, "ww_sha256"), (D, "D_sha256")):
        assert _sha(a) == g[key].tobytes(), "regenerated %s differs from the golden's" % key
    assert np.array_equal(y, g["y"])
    full = g["idx"].shape[2] == 0
    idx = (np.broadcast_to(np.arange(p["nv"], dtype=np.int64), (p["n"], 2, p["nv"])).copy()
           if full else g["idx"].astype(np.int64))
    return dict(X=X, y=y, ww=ww, D=D, idx=idx, full=full, C=p["C"], nb=idx.shape[2],
                scores=g["scores"], good=g["good"])


def agree(got, near, ref, nb):
    """Scores equal to the reference's bit for bit, or differing only where
    near ties were flagged: |got - ref| <= (near ties of the two evaluations) / nb.
    near: (n, 2) counts.  Returns the indices that differ (all flagged)."""
    diff = []
    for j in range(len(ref)):
        same = (np.isnan(got[j]) and np.isnan(ref[j])) or got[j] == ref[j]
        if same:
            continue
        diff.append(j)
        nt = int(near[j][0]) + int(near[j][1])
        assert nt > 0, "update %d: score %r != reference %r with no near tie flagged" % (j, got[j], ref[j])
        assert abs(got[j] - ref[j]) <= nt / nb + 1e-12, (j, got[j], ref[j], nt)
    return diff
