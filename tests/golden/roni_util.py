"""Load a RONI golden (tests/golden/gen_roni_goldens.py): inputs + the
reference's scores.  Large validation sets are regenerated from the case seed
and checked against the stored SHA-256."""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def names():
    return sorted(json.load(open(os.path.join(HERE, "roni_cases.json"))))


def load(name):
    g = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    if "Xv" in g.files:
        Xv = g["Xv"]
    else:
        import gen_roni_goldens as G  # make_case only; never touches the reference
        Xv = G.make_case(**G.CASES[name])[0]
    assert hashlib.sha256(np.ascontiguousarray(Xv).tobytes()).digest() == g["Xv_sha256"].tobytes(), \
        "regenerated validation set differs from the golden's"
    return Xv, g["yv"], g["ww"], g["deltas"], g["scores"]
