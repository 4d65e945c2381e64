"""MI355X parity of the torch-path RONI verifier (SURVEY.md §8(f) row 4 widened
to the mnist / lfw softmax models): client_obj.roni
(ML/Pytorch/client_obj.py:100-112) with the SoftmaxModel layout
(softmax_model.py:7-24) and getTrainErr's last-mini-batch argmax error
(client.py:136-144).

PINNED by the reference itself: the goldens
(tests/golden/gen_roni_softmax_goldens.py) are the reference's Client +
SoftmaxModel run in torch fp32 on the CPU; every update's two last batches are
recorded.  The GPU scores must equal the reference's, or differ only where
the GPU flags a near tie of torch's fp32 sgemm rounding -- and be bit-exact
against the C restatement oracle/roni_oracle.c, near-tie counts included.
Both entries: bk_roni_softmax_batches* (the reference's batch semantics) and
bk_roni_softmax* (one batch holding the whole set)."""
import numpy as np
import pytest

import rsm_util as RSM

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _case(nv, din, C, n, seed, nan=False, ties=False):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((nv, din)).astype(np.float32)
    if ties:
        X[: nv // 4] = 0.0  # every logit = its bias: exact ties between equal biases
    W = rng.standard_normal((C, din)) * 0.05
    b = rng.standard_normal(C) * 0.1
    if ties:
        b[:] = 0.25
    y = np.argmax(X.astype(np.float64) @ W.T + b, 1).astype(np.int32)
    flip = rng.random(nv) < 0.2
    y[flip] = (y[flip] + 1) % C
    ww = np.concatenate([W.ravel(), b])
    D = rng.standard_normal((n, ww.size)) * 10.0 ** rng.integers(-4, 0, size=(n, 1))
    if nan:
        D[0, 3] = np.nan
        D[-1, -1] = np.inf
    return X, y, ww, D


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _full(engine, X, y, C, ww, D):
    from biscotti_amd._lib import check, lib
    nv, din = X.shape
    n, d = D.shape
    tX, ty, tw, tD = _t(X), _t(y), _t(ww), _t(D)
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    nt = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    check(lib().bk_roni_softmax_device(engine.ctx, tX.data_ptr(), nv, din, din, ty.data_ptr(), C,
                                       tw.data_ptr(), tD.data_ptr(), n, d, out.data_ptr(),
                                       nt.data_ptr()))
    engine.synchronize()
    return out.cpu().numpy(), nt.cpu().numpy()


def _batches(engine, X, y, C, ww, D, idx):
    from biscotti_amd._lib import check, lib
    nv, din = X.shape
    n, d = D.shape
    tX, ty, tw, tD, ti = _t(X), _t(y), _t(ww), _t(D), _t(idx.astype(np.int64))
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    nt = torch.empty((n, 2), dtype=torch.int32, device="cuda")
    check(lib().bk_roni_softmax_batches_device(engine.ctx, tX.data_ptr(), nv, din, din,
                                               ty.data_ptr(), C, tw.data_ptr(), tD.data_ptr(), n,
                                               d, ti.data_ptr(), idx.shape[2], out.data_ptr(),
                                               nt.data_ptr()))
    engine.synchronize()
    return out.cpu().numpy(), nt.cpu().numpy()


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


@pytest.mark.parametrize("name", RSM.names())
def test_roni_softmax_reference_goldens(engine, oracle, name):
    c = RSM.load(name)
    got, nt = _batches(engine, c["X"], c["y"], c["C"], c["ww"], c["D"], c["idx"])
    want, wnt = oracle.roni_softmax_batches(c["X"], c["y"], c["C"], c["ww"], c["D"], c["idx"])
    assert np.array_equal(_bits(got), _bits(want))
    assert np.array_equal(nt, wnt)
    RSM.agree(got, nt, c["scores"], c["nb"])  # == the reference, or flagged
    if c["full"]:
        gf, ntf = _full(engine, c["X"], c["y"], c["C"], c["ww"], c["D"])
        assert np.array_equal(_bits(gf), _bits(got))
        assert np.all(ntf[0] == nt[:, 0]) and np.array_equal(ntf[1:], nt[:, 1])


@pytest.mark.parametrize("nv,din,C,n,kw", [
    (6000, 784, 10, 100, {}),            # mnist: a client's shard, a verifier's batch
    (1000, 784, 10, 1, {}),              # the Go verifier scores one update per call
    (777, 8742, 12, 5, {}),              # lfw's softmax (12 x 8,743)
    (3000, 24, 2, 33, {}),               # 2 classes
    (513, 100, 10, 7, {"nan": True}),    # NaN / inf updates: NaN logits win argmax
    (640, 64, 5, 9, {"ties": True}),     # exact logit ties: the first maximum
    (1, 1, 3, 2, {}),
    # the GEMM layout: 8 column tiles (the XCD-mapped grid), C = 16 (8 models
    # a tile), C = 3 (42 models a tile, 2 padding columns), a ragged d_in
    (500, 300, 10, 95, {}),
    (300, 129, 16, 63, {}),
    (257, 65, 3, 200, {"nan": True}),
    # r6 norm kernels: 16 samples / 512 features a chunk (k_roni_xnorm),
    # 16 columns / 256 features a chunk (k_roni_wnorm), ragged at every edge
    (17, 513, 10, 3, {}),
    (33, 1100, 4, 40, {}),
    (16, 256, 16, 1, {}),
])
def test_roni_softmax_full_set_vs_oracle(engine, oracle, nv, din, C, n, kw):
    X, y, ww, D = _case(nv, din, C, n, nv + din + C + n, **kw)
    want, wnt = oracle.roni_softmax(X, y, C, ww, D, near_ties=True)
    got, nt = _full(engine, X, y, C, ww, D)
    assert np.array_equal(_bits(got), _bits(want)), (got[:8], want[:8])
    assert np.array_equal(nt, wnt)


@pytest.mark.parametrize("nv,din,C,n,nb,kw", [
    (6000, 784, 10, 100, 10, {}),        # Biscotti: batch_size 10 (honest.go:47)
    (1003, 784, 10, 12, 3, {}),          # a ragged last batch
    (300, 8742, 12, 4, 10, {}),          # lfw
    (500, 300, 16, 9, 37, {}),           # C = 16 (every thread a logit), 5 sample tiles
    (200, 24, 2, 33, 8, {}),
    (513, 100, 10, 7, 10, {"nan": True}),
    (640, 64, 5, 9, 16, {"ties": True}),
    (50, 1, 3, 3, 1, {}),
])
def test_roni_softmax_batches_vs_oracle(engine, oracle, nv, din, C, n, nb, kw):
    X, y, ww, D = _case(nv, din, C, n, 7 * nv + din + C + n, **kw)
    rng = np.random.default_rng(nv + nb)
    idx = np.stack([np.stack([rng.permutation(nv)[:nb], rng.permutation(nv)[:nb]])
                    for _ in range(n)])
    want, wnt = oracle.roni_softmax_batches(X, y, C, ww, D, idx)
    got, nt = _batches(engine, X, y, C, ww, D, idx)
    assert np.array_equal(_bits(got), _bits(want)), (got[:8], want[:8])
    assert np.array_equal(nt, wnt)


def test_roni_softmax_batches_bad_index(engine):
    """A device-side index outside [0, nv): that update's score is NaN and its
    near ties -1, nothing read out of range; the host form returns BK_EINVAL."""
    from biscotti_amd.roni import SoftmaxRONIValidator
    X, y, ww, D = _case(100, 20, 4, 3, 1)
    idx = np.zeros((3, 2, 5), dtype=np.int64)
    idx[1, 1, 2] = 100
    idx[2, 0, 0] = -1
    got, nt = _batches(engine, X, y, 4, ww, D, idx)
    assert np.isfinite(got[0]) and np.isnan(got[1]) and np.isnan(got[2])
    assert nt[0].min() >= 0 and nt[1].tolist() == [-1, -1] and nt[2].tolist() == [-1, -1]
    v = SoftmaxRONIValidator(X, y, 4, engine=engine)
    with pytest.raises(ValueError):
        v.scores(ww, D, idx=idx)


def test_roni_softmax_validator(engine, oracle):
    """The verifyUpdate shape (the shard once, host updates): the reference's
    batch semantics by default (two fresh last batches per update), the whole
    set with batch_size=None; the verdicts (main.go:205-226: reject when the
    score exceeds 0.02)."""
    from biscotti_amd.krum import Update
    from biscotti_amd.roni import RONI_THRESHOLD, SoftmaxRONIValidator
    X, y, ww, D = _case(2000, 784, 10, 12, 5)
    D[8:] *= 1e3 / np.maximum(1e-30, np.abs(D[8:]).max())  # poisoned: large updates
    v = SoftmaxRONIValidator(X, y, 10, engine=engine, seed=3)
    idx = SoftmaxRONIValidator(X, y, 10, engine=engine, seed=3).draw_batches(len(D))
    assert idx.shape == (12, 2, 10) and np.all(idx < 2000)
    got = v.scores(ww, D)
    want, wnt = oracle.roni_softmax_batches(X, y, 10, ww, D, idx)
    assert np.array_equal(_bits(got), _bits(want))
    assert np.array_equal(v.last_near_ties, wnt)
    vf = SoftmaxRONIValidator(X, y, 10, engine=engine, batch_size=None)
    wf = oracle.roni_softmax(X, y, 10, ww, D)
    assert np.array_equal(_bits(vf.scores(ww, D)), _bits(wf))
    assert vf.roni(ww, D[3]) == wf[3]
    ups = [Update(SourceID=i, NoisedDelta=D[i]) for i in range(len(D))]
    assert np.array_equal(vf.verify_updates(ups, ww), ~(wf > RONI_THRESHOLD))
    with pytest.raises(ValueError):
        v.scores(ww[:-1], D[:, :-1])
