"""CPU: the RONI oracle (oracle/roni_oracle.c) against the goldens produced by
the reference roni (ML/code/logistic_validator.py:22-33; gen_roni_goldens.py):
scores bit-exact.  No GPU."""
import numpy as np
import pytest

import roni_util as RU


@pytest.mark.parametrize("name", RU.names())
def test_roni_oracle_matches_reference_goldens(oracle, name):
    Xv, yv, ww, deltas, want = RU.load(name)
    got = oracle.roni(Xv, yv, ww, deltas)
    assert np.array_equal(got.view(np.int64), want.view(np.int64)), (name, got, want)


def test_roni_oracle_semantics():
    from oracle import oracle as O
    Xv = np.array([[1.0, 0.0], [0.0, 0.0], [1.0, 1.0]])
    yv = np.array([1.0, 0.0, -1.0])
    # row 1 dots to 0: sign 0 == label 0 (no error); NaN weights -> every row errs
    s = O.roni(Xv, yv, np.array([1.0, 0.0]), np.array([[0.0, 0.0], [np.nan, 0.0], [-2.0, 0.0]]))
    assert s[0] == 0.0
    assert s[1] == 3 / 3 - 1 / 3
    assert s[2] == 1 / 3 - 1 / 3  # w = [-1, 0]: row 0 now wrong, row 2 now right


# ---- the torch-path (softmax) RONI: the oracle against the reference's own
#      Client.updateModel / getTrainErr + SoftmaxModel (gen_roni_softmax_goldens.py)
import rsm_util as RSM  # noqa: E402


@pytest.mark.parametrize("name", RSM.names())
def test_softmax_roni_oracle_matches_reference_goldens(oracle, name):
    """Scores equal the reference's bit for bit, or differ only where a near
    tie of torch's fp32 sgemm rounding is flagged (none differ today); the
    reference's per-evaluation correct counts are reproduced the same way."""
    c = RSM.load(name)
    sc, near = oracle.roni_softmax_batches(c["X"], c["y"], c["C"], c["ww"], c["D"], c["idx"])
    assert RSM.agree(sc, near, c["scores"], c["nb"]) == []
    if c["full"]:  # one batch = the whole set: the full-set restatement agrees too
        sf, ntf = oracle.roni_softmax(c["X"], c["y"], c["C"], c["ww"], c["D"], near_ties=True)
        assert np.array_equal(sf.view(np.int64), sc.view(np.int64))
        assert np.all(ntf[1:] == near[:, 1]) and np.all(ntf[0] == near[:, 0])


def test_softmax_roni_oracle_near_tie_semantics():
    """Exact logit ties are near ties; a clear winner is not; NaN logits are."""
    from oracle import oracle as O
    X = np.array([[0.0, 0.0], [1.0, 0.0]], dtype=np.float32)
    y = np.array([0, 0], dtype=np.int32)
    W = np.array([[1.0, 0.0], [0.0, 0.0]])
    b = np.array([0.5, 0.5])  # sample 0: logits tie (0.5, 0.5); sample 1: 1.5 vs 0.5
    ww = np.concatenate([W.ravel(), b])
    D = np.zeros((2, 6))
    D[1, 0] = np.nan
    idx = np.array([[[0, 1], [0, 1]], [[0, 1], [0, 1]]])
    sc, nt = O.roni_softmax_batches(X, y, 2, ww, D, idx)
    assert nt.tolist() == [[1, 1], [1, 2]]
    assert sc[0] == 0.0
    assert sc[1] == 0.0  # NaN logit 0 wins argmax: class 0 == label for both samples
