"""Golden vectors for the torch-path RONI verifier (SURVEY.md §8(f) row 4 on
the mnist / lfw softmax models), produced by the REFERENCE's own code on
repo-owned inputs.

Run once in the build container (the only place /root/reference exists):

    python tests/golden/gen_roni_softmax_goldens.py

What runs is the reference: ``Client.updateModel`` and ``Client.getTrainErr``
(ML/Pytorch/client.py:114-121, 136-144) on a ``SoftmaxModel``
(ML/Pytorch/softmax_model.py:7-24), in torch's fp32 on the CPU.  ``roni``
itself (ML/Pytorch/client_obj.py:100-112) is four lines of Python 2 in a
module that cannot be imported under Python 3 (``print "here"`` at :30), so
its body -- updateModel(ww); original = getTrainErr(); updateModel(ww + delta);
after = getTrainErr(); after - original -- is called here statement for
statement.  client.py imports torchvision (used only by Client.__init__, which
is bypassed: the Client is built with __new__) and the repo's ``datasets``
module (likewise only for __init__): both are stubbed in sys.modules.

The client's ``trainloader`` (client.py:20: DataLoader(trainset, batch_size,
shuffle=True)) is replaced by a loader with the same iteration semantics --
a fresh random permutation per pass, consecutive batches of batch_size, the
last one ragged -- that records the indices of each pass's LAST batch, the only
one getTrainErr's return value depends on (its loop overwrites pred and
labels).  So every update j yields the two batches the reference scored,
idx[j, 0] (`original`, model ww) and idx[j, 1] (`after`, model ww + delta_j),
and its score.  Samples are mnist-like: 0..255 pixels through torchvision's
ToTensor + Normalize((0.5,), (0.5,)) arithmetic in fp32.

Saved per case (.npz, numeric arrays, allow_pickle=False): y, idx (n x 2 x nb
int32; empty when one batch holds the whole set, whose order the error does
not depend on), scores, the reference's correct counts per evaluation, and the
SHA-256 of X, ww and the deltas, which tests regenerate with make_case (seeded
numpy PCG64) and check before use.
"""
import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/ML/Pytorch"


def make_case(seed, nv, din, C, n, batch, n_bad=0, nan=False, zero_rows=0, equal_bias=False):
    """Deterministic inputs (no reference code): X (nv, din) float32 as
    ToTensor + Normalize produce them, y (nv,) int labels, ww (C (din + 1),)
    fp64, deltas (n, C (din + 1)) fp64."""
    rng = np.random.default_rng(seed)
    proto = rng.random((C, din))
    y = rng.integers(0, C, nv)
    pix = np.clip(np.rint(255.0 * (0.55 * proto[y] + 0.45 * rng.random((nv, din)))), 0, 255)
    pix = pix.astype(np.uint8)
    # transforms.ToTensor (x / 255 in fp32) then Normalize((0.5,), (0.5,)): (x - 0.5) / 0.5
    X = (pix.astype(np.float32) / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5)
    if zero_rows:
        X[:zero_rows] = 0.0  # every logit = its bias
    flip = rng.random(nv) < 0.15  # label noise: some errors for every model
    y[flip] = (y[flip] + 1 + rng.integers(0, C - 1, int(flip.sum()))) % C
    W = (proto - proto.mean(0)) * (3.0 / np.sqrt(din)) + 0.02 * rng.standard_normal((C, din))
    b = 0.1 * rng.standard_normal(C)
    if equal_bias:
        b[:] = 0.125
    ww = np.concatenate([W.ravel(), b])
    D = rng.standard_normal((n, ww.size)) * 10.0 ** rng.integers(-4, -1, size=(n, 1))
    if n_bad:
        D[n - n_bad:] = -2.0 * ww + 0.05 * rng.standard_normal((n_bad, ww.size))  # flip the model
    if nan:
        D[0, 3] = np.nan
        D[min(1, n - 1), -1] = np.inf
    if n > 2:
        D[2] = 0.0  # a null update: its score is the difference of two batches' errors
    return X, y.astype(np.int32), ww, D


CASES = {
    # Biscotti's torch verifier: batch_size 10 (honest.go:47), a client shard of
    # 6,000 mnist samples (600 batches: the last one holds 10)
    "rsm_mnist_b10": dict(seed=11, nv=6000, din=784, C=10, n=100, batch=10, n_bad=20),
    # a ragged last batch (1,003 = 100 x 10 + 3)
    "rsm_mnist_ragged": dict(seed=12, nv=1003, din=784, C=10, n=12, batch=10, n_bad=3),
    # lfw's softmax (12 classes x 8,742 features, datasets.py get_num_features)
    "rsm_lfw": dict(seed=13, nv=400, din=8742, C=12, n=6, batch=10, n_bad=2),
    # batch_size >= the set: one batch holds every sample (the full-set entry)
    "rsm_full_set": dict(seed=14, nv=2000, din=784, C=10, n=30, batch=2000, n_bad=6),
    # NaN / inf updates: NaN logits win np.argmax
    "rsm_nan": dict(seed=15, nv=500, din=100, C=10, n=5, batch=10, nan=True),
    # 2 classes, 24 features (datasets.py's creditcard shape), batch 32
    "rsm_2class": dict(seed=16, nv=300, din=24, C=2, n=9, batch=32, n_bad=2),
    # exact logit ties (zero samples, equal biases): the first maximum
    "rsm_ties": dict(seed=17, nv=64, din=50, C=5, n=7, batch=16, zero_rows=40, equal_bias=True),
}


class ShuffleLoader:
    """DataLoader(trainset, batch_size, shuffle=True) iteration (client.py:20):
    a fresh permutation per pass, batches of batch_size, the last one ragged;
    records the last batch's sample indices."""

    def __init__(self, X, y, batch, seed):
        import torch
        self.torch = torch
        self.X, self.y, self.batch = X, y.astype(np.int64), batch
        self.g = np.random.default_rng(seed)
        self.last = None

    def __iter__(self):
        perm = self.g.permutation(len(self.X))
        for b0 in range(0, len(perm), self.batch):
            rows = perm[b0:b0 + self.batch]
            self.last = rows.copy()
            yield {"image": self.torch.from_numpy(self.X[rows]),
                   "label": self.torch.from_numpy(self.y[rows])}


def load_reference():
    tv = types.ModuleType("torchvision")  # only Client.__init__ uses it (bypassed)
    tvt = types.ModuleType("torchvision.transforms")
    tv.transforms = tvt
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tvt
    sys.modules["datasets"] = types.ModuleType("datasets")  # only Client.__init__ uses it
    sys.dont_write_bytecode = True
    mods = {}
    for name in ("softmax_model", "client"):
        spec = importlib.util.spec_from_file_location("ref_" + name, os.path.join(REF, name + ".py"))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        mods[name] = m
    return mods["client"], mods["softmax_model"]


def sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), dtype=np.uint8)


def main():
    client, softmax_model = load_reference()
    manifest = {}
    for name, p in CASES.items():
        X, y, ww, D = make_case(**p)
        n, C, din, nv = p["n"], p["C"], p["din"], p["nv"]
        c = client.Client.__new__(client.Client)
        c.model = softmax_model.SoftmaxModel(din, C)
        c.trainloader = ShuffleLoader(X, y, p["batch"], p["seed"] + 1000)
        scores, idx, good = [], [], []
        for j in range(n):
            # client_obj.roni(ww, delta), ML/Pytorch/client_obj.py:100-112
            weights = np.array(ww)
            update = np.array(D[j])
            c.updateModel(weights)
            original = c.getTrainErr()
            i0 = c.trainloader.last
            c.updateModel(weights + update)
            after = c.getTrainErr()
            i1 = c.trainloader.last
            scores.append(after - original)
            idx.append([i0, i1])
            nb = len(i0)
            good.append([int(round((1.0 - original) * nb)), int(round((1.0 - after) * nb))])
        idx = np.array(idx, dtype=np.int64)
        scores = np.array(scores, dtype=np.float64)
        full = p["batch"] >= nv  # one batch = every sample (a permutation of them)
        if full:
            assert all(np.array_equal(np.sort(r), np.arange(nv)) for r in idx.reshape(-1, nv))
        np.savez(os.path.join(HERE, name + ".npz"), y=y,
                 idx=np.zeros((n, 2, 0), np.int32) if full else idx.astype(np.int32),
                 scores=scores, good=np.array(good, dtype=np.int64), X_sha256=sha(X),
                 ww_sha256=sha(ww), D_sha256=sha(D))
        manifest[name] = dict(p, nb=int(idx.shape[2]),
                              n_nonzero=int(np.count_nonzero(scores)),
                              n_nan=int(np.isnan(scores).sum()))
        print(name, idx.shape, "scores[:6]", scores[:6], flush=True)
    with open(os.path.join(HERE, "roni_softmax_cases.json"), "w") as fp:
        json.dump(manifest, fp, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
