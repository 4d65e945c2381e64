"""MI355X parity of the RONI verifier through the C ABI:

* every golden produced by the reference roni (logistic_validator.py:22-33):
  scores bit-exact, through the device entry and the host entry
  (bk_roni_set_validation + bk_roni, the verifyUpdate shape);
* larger shapes against the CPU oracle (nv up to 200k, n up to 512);
* RONIValidator's verdicts (main.go:205-226) and argument errors.
"""
import numpy as np
import pytest

import roni_util as RU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()


def _roni_device(engine, Xv, yv, ww, deltas):
    from biscotti_amd._lib import check, lib
    n, d = deltas.shape
    tX, ty, tw, tD = _dev(Xv), _dev(yv), _dev(ww), _dev(deltas)
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    check(lib().bk_roni_device(engine.ctx, tX.data_ptr(), Xv.shape[0], d, d, ty.data_ptr(),
                               tw.data_ptr(), tD.data_ptr(), n, d, out.data_ptr()))
    engine.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", RU.names())
def test_roni_goldens_device(engine, name):
    Xv, yv, ww, deltas, want = RU.load(name)
    got = _roni_device(engine, Xv, yv, ww, deltas)
    assert np.array_equal(got.view(np.int64), want.view(np.int64)), (name, got, want)


@pytest.mark.parametrize("name", RU.names())
def test_roni_goldens_host_validator(engine, name):
    from biscotti_amd.roni import RONIValidator
    Xv, yv, ww, deltas, want = RU.load(name)
    v = RONIValidator(Xv, yv, engine=engine)
    got = v.scores(ww, deltas)
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
    # the Go verifier scores one update per call (honest.go:598-629)
    assert v.roni(ww, deltas[-1]) == want[-1]


@pytest.mark.parametrize("nv,d,n", [(200_000, 25, 16), (4096, 25, 512), (3000, 785, 33),
                                    (1, 1, 1), (1025, 1024, 2), (777, 25, 15), (778, 25, 16),
                                    # r3b: no cap on d (the MFMA form keeps no model in LDS)
                                    (2000, 7850, 9), (513, 3001, 130),
                                    # r6: the register kernel (d <= 32) at its edges
                                    # and the LDS kernel just past it
                                    (5000, 32, 200), (3001, 29, 129), (70, 4, 3),
                                    (1000, 5, 640), (999, 33, 64), (85_000, 25, 512)])
def test_roni_vs_oracle(engine, oracle, nv, d, n):
    rng = np.random.default_rng(nv + d + n)
    Xv = np.hstack([np.ones((nv, 1)), rng.standard_normal((nv, d - 1))]) if d > 1 else \
        np.ones((nv, 1))
    yv = np.where(rng.standard_normal(nv) > 0, 1.0, -1.0)
    ww = rng.standard_normal(d)
    deltas = rng.standard_normal((n, d)) * 10.0 ** rng.integers(-3, 1, size=(n, 1))
    want = oracle.roni(Xv, yv, ww, deltas)
    got = _roni_device(engine, Xv, yv, ww, deltas)
    assert np.array_equal(got.view(np.int64), want.view(np.int64))


def test_roni_verdicts_and_errors(engine):
    from biscotti_amd.krum import Update
    from biscotti_amd.roni import RONI_THRESHOLD, RONIValidator
    Xv, yv, ww, deltas, want = RU.load("roni_credit_like")
    v = RONIValidator(Xv, yv, engine=engine)
    ups = [Update(SourceID=i, NoisedDelta=deltas[i]) for i in range(len(deltas))]
    verdicts = v.verify_updates(ups, ww)
    assert np.array_equal(verdicts, ~(want > RONI_THRESHOLD))
    assert verdicts[:8].all() and not verdicts[8:].any()  # the 4 poisoned updates are rejected
    assert all(v.verify_update(u, ww) == bool(verdicts[i]) for i, u in enumerate(ups))
    assert RONIValidator(Xv, yv, engine=engine, priv_prob=0.1).verify_update(ups[-1], ww)
    with pytest.raises(ValueError):
        v.scores(ww[:-1], deltas[:, :-1])
