"""MI355X parity of the §8(f) rows 2-3 kernels (through the C ABI) against the
CPU oracle (oracle/aggregate_oracle.c), bit-exact:

* K4' block aggregation  global += X[idx[0]] + ... (honest.go:360-375), device
  and host entries, create_block end to end (stakes + gradient);
* K5  quantised int64 sum (kyber.go:698-757) incl. NaN/Inf/out-of-range,
  -0.0, truncation toward zero, int64 wrap, precision 0..18, fp32 input;
* K6  noise application (main.go:1524-1537, 1606-1653), k = 0..9, in place,
  odd d / misaligned rows;
* the BASELINE.json D batch at full size, checked on sampled columns.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402


def _rand(n, d, seed, spread=True):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d))
    if spread:
        X *= 10.0 ** rng.integers(-6, 3, size=(n, 1))
    return X


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n,d,ld,m,dtype", [
    (5, 1, 1, 3, "f64"), (9, 33, 33, 5, "f64"), (64, 1001, 1003, 40, "f64"),
    (100, 7850, 7850, 70, "f64"), (37, 4096, 4096, 37, "f32"), (20, 517, 520, 1, "f64"),
])
def test_aggregate_device_vs_oracle(engine, oracle, n, d, ld, m, dtype):
    rng = np.random.default_rng(n * 7 + d)
    Xp = _rand(n, ld, n + d)
    if dtype == "f32":
        Xp = Xp.astype(np.float32)
    X = Xp[:, :d]
    idx = rng.integers(0, n, size=m).astype(np.int64)  # any order, duplicates allowed
    g0 = _rand(1, d, 3)[0]
    want = oracle.aggregate(X.astype(np.float64), idx, g0)
    tX, tI, tG = _dev(Xp), _dev(idx), _dev(g0)
    dt = _lib.BK_F32 if dtype == "f32" else _lib.BK_F64
    engine.aggregate_device_ptr(tX.data_ptr(), dt, n, d, ld, tI.data_ptr(), m, tG.data_ptr())
    engine.synchronize()
    got = tG.cpu().numpy()
    assert np.array_equal(got.view(np.int64), want.view(np.int64))


def test_aggregate_host_entry_and_m0(engine, oracle):
    X = _rand(30, 257, 5)
    idx = np.array([29, 0, 7, 7, 13], dtype=np.int64)
    g = _rand(1, 257, 6)[0]
    want = oracle.aggregate(X, idx, g)
    got = engine.aggregate(X, idx, g.copy())
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
    assert np.array_equal(engine.aggregate(X, np.array([], dtype=np.int64), g.copy()), g)
    with pytest.raises(ValueError):
        engine.aggregate(X, np.array([30], dtype=np.int64), g.copy())


def test_create_block_end_to_end(engine, oracle):
    from biscotti_amd.aggregate import STAKE_UNIT, create_block
    from biscotti_amd.krum import Update
    d = 1003
    ups = [Update(SourceID=s, Delta=_rand(1, d, s)[0], Accepted=(s % 3 != 0))
           for s in (4, 1, 9, 6, 2, 8, 5)]
    stake = {4: 100, 9: 50}
    g0 = _rand(1, d, 77)[0]
    got = create_block(g0, ups, stake, engine=engine)
    acc = [i for i, u in enumerate(ups) if u.Accepted]
    want = oracle.aggregate(np.stack([u.Delta for u in ups]), acc, g0)
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
    assert stake[4] == 100 + STAKE_UNIT and stake[9] == 50 - STAKE_UNIT
    assert stake[6] == -STAKE_UNIT and stake[1] == STAKE_UNIT


def _special(X, prec):
    X = X.copy()
    X[0, 0] = np.nan
    X[0, 1] = np.inf
    X[1, 1] = -np.inf
    X[1, 2] = -0.0
    X[2, 3] = 9.3e18 / 10.0 ** prec        # out of int64 range after scaling
    X[3, 4] = 9.2e18 / 10.0 ** prec        # in range; two of them wrap the sum
    X[4, 4] = 9.2e18 / 10.0 ** prec
    X[2, 5] = -1.99999 / 10.0 ** prec      # truncation toward zero -> -1
    return X


@pytest.mark.parametrize("prec", [0, 4, 9, 18])
@pytest.mark.parametrize("n,d,m", [(8, 7, 5), (70, 1001, 64), (100, 7850, 70)])
def test_quantized_sum_vs_oracle(engine, oracle, prec, n, d, m):
    X = _special(_rand(n, d, prec + d), prec)
    idx = np.concatenate([np.arange(min(5, n)), np.random.default_rng(d).integers(0, n, m - min(5, n))]).astype(np.int64)
    want_s, want_f = oracle.qsum(X, idx, prec)
    tX, tI = _dev(X), _dev(idx)
    s = torch.empty(d, dtype=torch.int64, device="cuda")
    sf = torch.empty(d, dtype=torch.float64, device="cuda")
    engine.quantized_sum_ptr(tX.data_ptr(), _lib.BK_F64, n, d, d, tI.data_ptr(), m, prec,
                             s.data_ptr(), sf.data_ptr())
    engine.synchronize()
    assert np.array_equal(s.cpu().numpy(), want_s)
    assert np.array_equal(sf.cpu().numpy().view(np.int64), want_f.view(np.int64))


def test_quantized_sum_fp32_and_mirror(engine, oracle):
    from biscotti_amd.aggregate import quantized_sum
    X = _rand(50, 3000, 9).astype(np.float32)
    idx = np.arange(0, 50, 2)
    want = oracle.qsum(X.astype(np.float64), idx, 4)
    got = quantized_sum(X, idx, 4, engine=engine)
    assert np.array_equal(got[0], want[0])
    assert np.array_equal(got[1].view(np.int64), want[1].view(np.int64))


def test_quantized_sum_bad_precision(engine):
    t = torch.zeros((2, 2), dtype=torch.float64, device="cuda")
    i = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.empty(2, dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError):
        engine.quantized_sum_ptr(t.data_ptr(), _lib.BK_F64, 2, 2, 2, i.data_ptr(), 1, 19,
                                 s.data_ptr())


@pytest.mark.parametrize("n,d,ld,k", [(3, 17, 17, 0), (3, 17, 17, 1), (5, 1001, 1003, 3),
                                      (16, 4096, 4096, 9), (2, 7850, 7851, 2)])
def test_noise_vs_oracle(engine, oracle, n, d, ld, k):
    rng = np.random.default_rng(k * 100 + d)
    Dp = rng.standard_normal((n, ld))
    N = rng.standard_normal((n, max(k, 1), ld)) * 1e-3
    N[0, 0, 1] = -0.0
    want = oracle.noise(Dp[:, :d], N[:, :k, :d])
    tD, tN = _dev(Dp), _dev(N)
    out = torch.full((n, ld), 7.0, dtype=torch.float64, device="cuda")
    engine.noise_apply_ptr(tD.data_ptr(), n, d, ld, tN.data_ptr(), k, ld, out.data_ptr(), ld)
    engine.synchronize()
    got = out.cpu().numpy()[:, :d]
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
    # in place (out aliases delta)
    engine.noise_apply_ptr(tD.data_ptr(), n, d, ld, tN.data_ptr(), k, ld, tD.data_ptr(), ld)
    engine.synchronize()
    assert np.array_equal(tD.cpu().numpy()[:, :d].view(np.int64), want.view(np.int64))


def test_noise_mirror_single_update(engine, oracle):
    from biscotti_amd.aggregate import apply_noise
    rng = np.random.default_rng(4)
    delta = rng.standard_normal(7850)
    noise = rng.standard_normal((3, 7850)) * 1e-2
    got = apply_noise(delta, noise, engine=engine)
    want = oracle.noise(delta[None], noise[None])[0]
    assert np.array_equal(got.view(np.int64), want.view(np.int64))


def test_full_size_D_sampled_columns(engine, oracle):
    """BASELINE.json config D (512 x 1,048,576 fp64) generated on the device:
    aggregation of the 359 rows in a shuffled order, quantised sum and noise,
    checked bit-exactly on 2048 sampled columns."""
    n, d = 512, 1 << 20
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 20261019, 153)
    rng = np.random.default_rng(0)
    idx = rng.permutation(n)[:359].astype(np.int64)
    cols = np.sort(rng.choice(d, 2048, replace=False))
    tI = _dev(idx)
    g = torch.zeros(d, dtype=torch.float64, device="cuda")
    engine.aggregate_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, tI.data_ptr(), 359,
                                g.data_ptr())
    s = torch.empty(d, dtype=torch.int64, device="cuda")
    sf = torch.empty(d, dtype=torch.float64, device="cuda")
    engine.quantized_sum_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, tI.data_ptr(), 359, 4,
                             s.data_ptr(), sf.data_ptr())
    engine.synchronize()
    Xs = X[:, torch.from_numpy(cols).cuda()].cpu().numpy()
    want = oracle.aggregate(Xs, idx, np.zeros(len(cols)))
    assert np.array_equal(g.cpu().numpy()[cols].view(np.int64), want.view(np.int64))
    ws, wf = oracle.qsum(Xs, idx, 4)
    assert np.array_equal(s.cpu().numpy()[cols], ws)
    assert np.array_equal(sf.cpu().numpy()[cols].view(np.int64), wf.view(np.int64))
