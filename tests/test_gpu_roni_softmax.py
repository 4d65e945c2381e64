"""MI355X parity of the torch-path RONI verifier (SURVEY.md §8(f) row 4 widened
to the mnist / lfw softmax models): client_obj.roni
(ML/Pytorch/client_obj.py:100-112) with the SoftmaxModel layout
(softmax_model.py:19-24) and getTrainErr's argmax error (client.py:131-139).

PARITY UNPINNED by the reference itself: client_obj.py is Python 2 and its
client / dataset modules (torchvision, the mnist files) are absent, so no
reference output exists; the GPU is checked BIT FOR BIT against the committed
C restatement oracle/roni_oracle.c:oracle_roni_softmax (whose numpy form is in
its header), on mnist's shape (10 classes x 785 = 7,850 parameters), lfw's
(12 x 8,743) and edge cases (2 classes, NaN updates, label ties)."""
import numpy as np
import pytest

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


def _device(engine, X, y, C, ww, D):
    from biscotti_amd._lib import check, lib
    nv, din = X.shape
    n, d = D.shape
    tX = torch.from_numpy(X).cuda()
    ty = torch.from_numpy(y).cuda()
    tw = torch.from_numpy(ww).cuda()
    tD = torch.from_numpy(np.ascontiguousarray(D)).cuda()
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    check(lib().bk_roni_softmax_device(engine.ctx, tX.data_ptr(), nv, din, din, ty.data_ptr(), C,
                                       tw.data_ptr(), tD.data_ptr(), n, d, out.data_ptr()))
    engine.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("nv,din,C,n,kw", [
    (6000, 784, 10, 100, {}),            # mnist: a client's shard, a verifier's batch
    (1000, 784, 10, 1, {}),              # the Go verifier scores one update per call
    (777, 8742, 12, 5, {}),              # lfw's softmax (12 x 8,743)
    (3000, 24, 2, 33, {}),               # 2 classes
    (513, 100, 10, 7, {"nan": True}),    # NaN / inf updates: NaN logits win argmax
    (640, 64, 5, 9, {"ties": True}),     # exact logit ties: the first maximum
    (1, 1, 3, 2, {}),
    # r3b GEMM layout: 8 column tiles (the XCD-mapped grid), C = 16 (8 models
    # a tile), C = 3 (42 models a tile, 2 padding columns), a ragged d_in
    (500, 300, 10, 95, {}),
    (300, 129, 16, 63, {}),
    (257, 65, 3, 200, {"nan": True}),
])
def test_roni_softmax_vs_oracle(engine, oracle, nv, din, C, n, kw):
    X, y, ww, D = _case(nv, din, C, n, nv + din + C + n, **kw)
    want = oracle.roni_softmax(X, y, C, ww, D)
    got = _device(engine, X, y, C, ww, D)
    assert np.array_equal(got.view(np.int64), want.view(np.int64)), (got[:8], want[:8])


def test_roni_softmax_validator(engine, oracle):
    """The verifyUpdate shape (validation set once, host updates) and the
    verdicts (main.go:205-226: reject when the score exceeds 0.02)."""
    from biscotti_amd.krum import Update
    from biscotti_amd.roni import RONI_THRESHOLD, SoftmaxRONIValidator
    X, y, ww, D = _case(2000, 784, 10, 12, 5)
    D[8:] *= 1e3 / np.maximum(1e-30, np.abs(D[8:]).max())  # poisoned: large updates
    want = oracle.roni_softmax(X, y, 10, ww, D)
    v = SoftmaxRONIValidator(X, y, 10, engine=engine)
    got = v.scores(ww, D)
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
    assert v.roni(ww, D[3]) == want[3]
    ups = [Update(SourceID=i, NoisedDelta=D[i]) for i in range(len(D))]
    assert np.array_equal(v.verify_updates(ups, ww), ~(want > RONI_THRESHOLD))
    with pytest.raises(ValueError):
        v.scores(ww[:-1], D[:, :-1])
