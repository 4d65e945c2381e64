"""Golden vectors for the RONI verifier, produced by the
REFERENCE ``roni`` on repo-owned inputs.

Run once in the build container (the only place /root/reference exists):

    python tests/golden/gen_roni_goldens.py

``roni(ww, delta)`` (ML/code/logistic_validator.py:22-33, bound as pyRoniFunc
at DistSys/honest.go:235-243 and called per update by verifyUpdate,
honest.go:598-629) reads the module-level validation set that the module body
loads through ``utils.load_dataset("credittest")`` (:6-7).  The dataset is not
shipped (.MISSING_LARGE_BLOBS), so each case imports the module afresh with a
stub ``utils`` that returns the case's synthetic validation set, shaped like
the creditcard one (utils.py:86-117: a bias column of ones, standardised
features, int labels in {-1, +1}).  Only the reference's outputs on our inputs
are saved (.npz, numeric arrays, allow_pickle=False).

Saved per case: yv (float64 copies of the int labels), ww, deltas (n x d),
scores[i] = roni(ww, deltas[i]), and Xv -- or, for large validation sets, only
Xv_sha256: tests regenerate Xv with make_case (seeded numpy PCG64) and check the
hash before use.
"""
import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/ML/code/logistic_validator.py"


def load_reference(Xv, yv, tag):
    stub = types.ModuleType("utils")
    stub.load_dataset = lambda name: {"X": Xv, "y": yv}
    sys.modules["utils"] = stub
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("ref_logistic_validator_%s" % tag, REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_case(seed, nv, d, n, n_bad, zero_rows=0, nan_update=False, label01=False):
    rng = np.random.default_rng(seed)
    feats = rng.standard_normal((nv, d - 1))
    Xv = np.hstack([np.ones((nv, 1)), feats])
    if zero_rows:
        Xv[:zero_rows] = 0.0  # sign(0) = 0 never equals a label: always an error
    wstar = rng.standard_normal(d)
    margin = Xv @ wstar + 0.5 * rng.standard_normal(nv)
    yv = np.where(margin > 0, 1, -1).astype(int)
    if label01:
        yv[yv == -1] = 0
    ww = wstar + 0.3 * rng.standard_normal(d)
    deltas = 1e-2 * rng.standard_normal((n, d))          # honest: small steps
    deltas[n - n_bad:] = -2.0 * ww + rng.standard_normal((n_bad, d))  # poisoned: flip the model
    if nan_update:
        deltas[0, 3] = np.nan
    deltas[1] = 0.0                                      # a null update scores exactly 0
    return Xv, yv, ww, deltas


CASES = {
    # creditcard-shaped: d = 25, a validation split of a few thousand rows
    "roni_credit_like": dict(seed=1, nv=2000, d=25, n=12, n_bad=4),
    "roni_zero_rows": dict(seed=2, nv=777, d=25, n=6, n_bad=2, zero_rows=40),
    "roni_nan_update": dict(seed=3, nv=500, d=25, n=4, n_bad=1, nan_update=True),
    "roni_labels01": dict(seed=4, nv=1000, d=25, n=5, n_bad=2, label01=True),
    "roni_wide": dict(seed=5, nv=8192, d=100, n=64, n_bad=20),
    "roni_tiny": dict(seed=6, nv=3, d=2, n=3, n_bad=1),
}


def main():
    manifest = {}
    for name, p in CASES.items():
        Xv, yv, ww, deltas = make_case(**p)
        ref = load_reference(Xv, yv, name)
        scores = np.array([ref.roni(list(ww), list(deltas[i])) for i in range(len(deltas))],
                          dtype=np.float64)
        arrays = dict(yv=yv.astype(np.float64), ww=ww, deltas=deltas, scores=scores,
                      Xv_sha256=np.frombuffer(hashlib.sha256(Xv.tobytes()).digest(), np.uint8))
        if Xv.size <= 100_000:
            arrays["Xv"] = Xv
        np.savez(os.path.join(HERE, name + ".npz"), **arrays)
        manifest[name] = dict(p, scores=scores.tolist())
        print(name, scores)
    json.dump(manifest, open(os.path.join(HERE, "roni_cases.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
