"""Parity of the HIP path (libbk.so, through its C ABI) on an MI355X.

* every small golden (produced by the reference numpy krum, see
  tests/golden/gen_goldens.py): selected set bit-exact, scores within 1e-9 of
  the max score, mean within 1e-9 of the norm-wise scale;
* the BASELINE.json configs at full size (C, D f=153 / f=256, E fp32) against
  their goldens, with the batch generated on the device;
* the CPU oracle on shapes and layouts the goldens do not cover (ld padding,
  misaligned base, fp32, n not a multiple of 64, tiny/huge k);
* the sharded decomposition (partial Grams summed) == the unsharded call;
* run-to-run bitwise determinism; argument errors; the GPU generator == CPU.
"""
import numpy as np
import pytest

import golden_util as GU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402


def _dev_run(engine, Xt, f, dtype=None):
    n, d = Xt.shape
    dt = _lib.BK_F32 if Xt.dtype == torch.float32 else _lib.BK_F64
    sel = torch.empty(n - f, dtype=torch.int64, device=Xt.device)
    sc = torch.empty(n, dtype=torch.float64, device=Xt.device)
    mean = torch.empty(d, dtype=torch.float64, device=Xt.device)
    engine.multikrum_device_ptr(Xt.data_ptr(), dt, n, d, Xt.stride(0), f, sel.data_ptr(),
                                sc.data_ptr(), mean.data_ptr())
    engine.synchronize()
    return sel.cpu().numpy(), sc.cpu().numpy(), mean.cpu().numpy()


@pytest.mark.parametrize("name", GU.small_cases())
def test_small_goldens(name, engine, oracle):
    X, p = GU.build_input(name, oracle)
    rec = GU.manifest()[name]
    if p["error"]:
        with pytest.raises(ValueError):
            engine.multikrum(X, p["f"])
        return
    g = GU.load(name)
    sel, sc, mean = engine.multikrum(X, p["f"])
    assert np.array_equal(sel, g["sel"]), (name, sel, g["sel"])
    GU.check_scores(sc, g, rel=1e-9)
    GU.check_mean(mean, g, rec)


@pytest.mark.parametrize("name", GU.large_cases())
def test_large_goldens_device_resident(name, engine):
    p = GU.C.case_params(name)
    n, d, f = p["n"], p["d"], p["f"]
    tdt = torch.float32 if p["dtype"] == "float32" else torch.float64
    dt = _lib.BK_F32 if p["dtype"] == "float32" else _lib.BK_F64
    X = torch.empty((n, d), dtype=tdt, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), dt, n, d, X.stride(0), 0, d, p["seed"], p["nbyz"],
                          p["mu_scale"], p["byz_scale"], p["sigma"], p["flags"])
    sel, sc, mean = _dev_run(engine, X, f)
    g = GU.load(name)
    assert np.array_equal(sel, g["sel"])
    GU.check_scores(sc, g, rel=1e-9)
    GU.check_mean(mean, g, GU.manifest()[name])
    # size-independent properties: m distinct ascending indices; every
    # selected score <= every rejected score
    assert len(np.unique(sel)) == n - f and np.all(np.diff(sel) > 0)
    rej = np.setdiff1d(np.arange(n), sel)
    assert np.max(sc[sel]) <= np.min(sc[rej])
    del X
    torch.cuda.empty_cache()


def test_gpu_generator_matches_cpu(engine, oracle):
    for (n, d, nbyz, flags, tdt, dt) in [(37, 1003, 5, 0, torch.float64, _lib.BK_F64),
                                         (100, 785, 30, 1, torch.float64, _lib.BK_F64),
                                         (64, 300, 20, 0, torch.float32, _lib.BK_F32)]:
        X = torch.empty((n, d + 3), dtype=tdt, device="cuda")  # padded ld
        engine.synth_fill_ptr(X.data_ptr(), dt, n, d, X.stride(0), 0, d, 77, nbyz, flags=flags)
        engine.synchronize()
        ref = oracle.synth(n, d, 77, nbyz, flags=flags,
                           dtype=np.float32 if tdt == torch.float32 else np.float64)
        got = X[:, :d].cpu().numpy()
        assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))
        # a column shard of the same batch
        Xs = torch.empty((n, 100), dtype=tdt, device="cuda")
        engine.synth_fill_ptr(Xs.data_ptr(), dt, n, 100, 100, 200, d, 77, nbyz, flags=flags)
        engine.synchronize()
        assert np.array_equal(Xs.cpu().numpy().view(np.uint8),
                              np.ascontiguousarray(ref[:, 200:300]).view(np.uint8))


@pytest.mark.parametrize("n,d,f,pad,dtype", [
    (1, 8, 0, 0, np.float64),      # n=1 -> invalid
    (2, 1, 1, 0, np.float64), (3, 7, 1, 1, np.float64), (64, 64, 20, 0, np.float64),
    (65, 129, 30, 2, np.float64), (128, 1000, 1, 0, np.float64), (200, 333, 198, 0, np.float64),
    (257, 2049, 77, 5, np.float32), (300, 40000, 90, 0, np.float32), (513, 4099, 153, 0, np.float64),
    (40, 100003, 12, 0, np.float64),
    # fp32 on K1 v3 (ld % 4 == 0): 32-column k-blocks, ragged tails, all-tail
    (129, 4100, 40, 3, np.float32), (700, 32804, 210, 0, np.float32), (64, 28, 20, 0, np.float32),
    (100, 7852, 30, 0, np.float32)])
def test_against_oracle(engine, oracle, n, d, f, pad, dtype):
    X = oracle.synth(n, d, 1000 + n + d, max(0, min(f, n)), dtype=dtype)
    if pad:
        Xp = np.zeros((n, d + pad), dtype=dtype)
        Xp[:, :d] = X
        Xv = Xp[:, :d]  # ld = d + pad (odd pads exercise the unaligned kernel variants)
    else:
        Xv = X
    if f < 1 or f >= n:
        with pytest.raises(ValueError):
            engine.multikrum(Xv, f)
        return
    sel, sc, mean = engine.multikrum(Xv, f)
    osel, osc, omean = oracle.krum(X, f)
    assert np.array_equal(sel, osel)
    scale = max(1e-300, np.max(np.abs(osc)))
    assert np.max(np.abs(sc - osc)) <= 1e-9 * scale
    mscale = np.max(np.mean(np.abs(X[osel].astype(np.float64)), axis=0))
    assert np.max(np.abs(mean - omean)) <= 1e-9 * mscale


def test_misaligned_device_pointer(engine, oracle):
    n, d, f = 70, 999, 20
    X = oracle.synth(n, d, 5, 20)
    buf = torch.zeros(n * d + 1, dtype=torch.float64, device="cuda")
    view = buf[1:].view(n, d)  # 8-B aligned, not 16-B: scalar-load kernels
    view.copy_(torch.from_numpy(X).cuda())
    sel, sc, mean = _dev_run(engine, view, f)
    osel, osc, omean = oracle.krum(X, f)
    assert np.array_equal(sel, osel)
    assert np.max(np.abs(mean - omean)) <= 1e-9 * np.max(np.abs(omean)) * 10


def test_odd_ld_device_rows(engine, oracle):
    """Device rows whose starts are not all 16-B aligned (odd ld): the
    direct-to-register K1 (k_gram v1).  Host input is re-staged with a padded
    ld and never takes this path."""
    n, d, f, ld = 90, 1003, 27, 1005
    X = oracle.synth(n, d, 6, f)
    buf = torch.zeros((n, ld), dtype=torch.float64, device="cuda")
    buf[:, :d] = torch.from_numpy(X).cuda()
    sel, sc, mean = _dev_run(engine, buf[:, :d], f)
    osel, osc, omean = oracle.krum(X, f)
    assert np.array_equal(sel, osel)
    assert np.max(np.abs(sc - osc)) <= 1e-9 * np.max(np.abs(osc))
    mscale = np.max(np.mean(np.abs(X[osel]), axis=0))
    assert np.max(np.abs(mean - omean)) <= 1e-9 * mscale


@pytest.mark.parametrize("n,d,f", [(16384, 40, 4915), (9001, 33, 1)])
def test_max_n(engine, oracle, n, d, f):
    """BK_MAX_N = 16384 updates (the row sort takes 128 KiB of LDS), and a
    ragged n just past 9000 with k = n - 3."""
    X = oracle.synth(n, d, 7 + n, f)
    sel, sc, mean = engine.multikrum(X, f)
    osel, osc, omean = oracle.krum(X, f)
    assert np.array_equal(sel, osel)
    assert np.max(np.abs(sc - osc)) <= 1e-9 * np.max(np.abs(osc))
    mscale = np.max(np.mean(np.abs(X[osel]), axis=0))
    assert np.max(np.abs(mean - omean)) <= 1e-9 * mscale


def test_deterministic_bitwise(engine):
    n, d, f = 512, 200003, 153
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 42, 153)
    a = _dev_run(engine, X, f)
    b = _dev_run(engine, X, f)
    for u, v in zip(a, b):
        assert np.array_equal(u.view(np.uint8), v.view(np.uint8))


def test_sharded_decomposition_equals_full(engine):
    """Packed partial Grams of column shards, summed, then finished == one
    unsharded call: the multi-GPU path's math on the real kernels."""
    from biscotti_amd.dist import all_shards
    n, d, f = 300, 50000, 90
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 9, 90)
    usz = int(_lib.lib().bk_upper_elems(n))
    acc = torch.zeros(usz, dtype=torch.float64, device="cuda")
    for c0, dl in all_shards(d, 4):
        U = torch.empty(usz, dtype=torch.float64, device="cuda")
        Xs = X[:, c0:c0 + dl]
        engine.gram_upper_ptr(Xs.data_ptr(), _lib.BK_F64, n, dl, X.stride(0), U.data_ptr())
        engine.synchronize()
        acc += U
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mean = torch.empty(d, dtype=torch.float64, device="cuda")
    engine.finish_ptr(acc.data_ptr(), X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(),
                      sc.data_ptr(), mean.data_ptr())
    engine.synchronize()
    fsel, fsc, fmean = _dev_run(engine, X, f)
    assert np.array_equal(sel.cpu().numpy(), fsel)
    s = sc.cpu().numpy()
    assert np.max(np.abs(s - fsc)) <= 1e-12 * np.max(np.abs(fsc))
    assert np.array_equal(mean.cpu().numpy(), fmean)
    # single-rank sharded entry (no communicator needed) == unsharded
    sel2 = torch.empty(n - f, dtype=torch.int64, device="cuda")
    engine.multikrum_sharded_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel2.data_ptr())
    engine.synchronize()
    assert np.array_equal(sel2.cpu().numpy(), fsel)


@pytest.mark.parametrize("n,d,f,nsh", [(300, 50000, 90, 4), (700, 65536, 210, 8)])
def test_sharded_decomposition_fp32(engine, oracle, n, d, f, nsh):
    """Config E's form (fp32 updates, d sharded over ranks): per-shard fp32 Grams
    (K1 v3, 32-column k-blocks) summed == the oracle on the exact fp64 widening."""
    from biscotti_amd.dist import all_shards
    X = torch.empty((n, d), dtype=torch.float32, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, 0, d, 11, f)
    usz = int(_lib.lib().bk_upper_elems(n))
    acc = torch.zeros(usz, dtype=torch.float64, device="cuda")
    for c0, dl in all_shards(d, nsh):
        U = torch.empty(usz, dtype=torch.float64, device="cuda")
        Xs = X[:, c0:c0 + dl]
        engine.gram_upper_ptr(Xs.data_ptr(), _lib.BK_F32, n, dl, X.stride(0), U.data_ptr())
        engine.synchronize()
        acc += U
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    mean = torch.empty(d, dtype=torch.float64, device="cuda")
    engine.finish_ptr(acc.data_ptr(), X.data_ptr(), _lib.BK_F32, n, d, d, f, sel.data_ptr(),
                      None, mean.data_ptr())
    engine.synchronize()
    Xh = X.cpu().numpy()
    osel, _, omean = oracle.krum(Xh, f)
    assert np.array_equal(sel.cpu().numpy(), osel)
    mscale = np.max(np.mean(np.abs(Xh[osel].astype(np.float64)), axis=0))
    assert np.max(np.abs(mean.cpu().numpy() - omean)) <= 1e-9 * mscale


def test_validator_end_to_end(engine, oracle):
    from biscotti_amd.krum import KRUMValidator, Update, get_krum_scores, krum, krum_mean
    X = oracle.synth(10, 25, 20261016, 2)
    v = KRUMValidator(engine=engine).initialize()
    v.UpdateList = [Update(SourceID=100 + i, NoisedDelta=X[i]) for i in range(10)]
    v.compute_scores()
    osel, osc, omean = oracle.krum(X, 5)  # clip = int(0.5 * 10)
    assert v.AcceptedList == osel.tolist()
    for i in range(10):
        assert v.check_if_accepted(100 + i) == (i in osel)
    assert np.array_equal(krum(X.tolist(), 2, engine), oracle.krum(X, 2)[0])
    sc = get_krum_scores(X, 8, engine)
    assert np.max(np.abs(sc - oracle.krum(X, 2)[1])) <= 1e-9 * np.max(np.abs(sc))
    s, m = krum_mean(X, 2, engine)
    assert np.array_equal(s, oracle.krum(X, 2)[0])


def test_timing_api(engine):
    n, d, f = 129, 4096, 30  # n > 128: the general chain (k_small takes n <= 128)
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 1, 30)
    engine.timing_enable(True)
    for _ in range(3):
        _dev_run(engine, X, f)
    t = engine.timing_read()
    engine.timing_enable(False)
    for k in ("k_gram", "k_reduce", "k_scores", "k_rank", "k_compact", "k_mean"):
        assert t[k]["count"] == 3 and t[k]["avg_ms"] > 0
    assert "k_transpose" not in t  # small n: k_scores reads the packed upper tiles


@pytest.mark.parametrize("deterministic", [False, True])
def test_rccl_exchange_single_rank(engine, deterministic):
    """The sharded entry with a real RCCL communicator (1 rank on this box):
    the all-reduce / all-gather + fixed-order sum must leave the result
    bitwise unchanged.  N > 1 runs are the driver's 8-GPU bench."""
    from biscotti_amd.krum import Engine, comm_unique_id
    e2 = Engine(0)
    e2.set_stream(torch.cuda.current_stream().cuda_stream)
    e2.comm_init(1, 0, comm_unique_id())
    e2.comm_set_mode(deterministic)
    n, d, f = 300, 70001, 90
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 13, 90)
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mean = torch.empty(d, dtype=torch.float64, device="cuda")
    e2.multikrum_sharded_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(),
                             sc.data_ptr(), mean.data_ptr())
    e2.synchronize()
    fsel, fsc, fmean = _dev_run(engine, X, f)
    assert np.array_equal(sel.cpu().numpy(), fsel)
    assert np.array_equal(sc.cpu().numpy(), fsc)
    assert np.array_equal(mean.cpu().numpy(), fmean)
    e2.close()


@pytest.mark.parametrize("n", [2, 3, 5, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512,
                               513, 777, 1023, 1024, 1025, 2049])
def test_exact_ties_bitwise(engine, oracle, n):
    """Integer-valued updates in {-1, 0, 1}: every Gram entry, distance and
    score is an exact integer, so the GPU must agree with the oracle BITWISE
    on the scores -- whatever the summation order -- and, with the heavy ties
    this makes in distances and in scores, on the selected set under the
    (value, index) total order (ties at the boundary go to the lower index)."""
    rng = np.random.default_rng(1000 + n)
    d = 40
    X = rng.integers(-1, 2, size=(n, d)).astype(np.float64)
    X[n // 2:n // 2 + max(1, n // 8)] = X[0]  # duplicated rows: zero distances, equal scores
    for f in sorted({1, max(1, n // 3), max(1, n - 3), n - 1}):
        if not 1 <= f < n:
            continue
        sel, sc, _ = engine.multikrum(X, f)
        osel, osc, _ = oracle.krum(X, f)
        assert np.array_equal(sel, osel), (n, f)
        assert np.array_equal(sc, osc), (n, f)


@pytest.mark.parametrize("n", [200, 2100, 4500])
def test_nan_and_inf_rows(engine, oracle, n):
    """NaN / Inf rows: NaN-aware score agreement with the oracle and the same
    selection (NaN sorts last, as in numpy).  n = 200 runs K2's lane-exchange
    sort, 2100 and 4500 the register-local one on transposed rows (16 keys
    per thread, 4096 / 8192 keys), where NaN distances sort as +inf and are
    put back at ranks n - #NaN .. n - 1."""
    rng = np.random.default_rng(5)
    X = rng.standard_normal((n, 64))
    X[7] = np.nan
    X[50, 3] = np.inf
    X[120] = -np.inf
    X[n - 3, 10] = np.nan
    for f in (n // 10, 3 * n // 10, 3 * n // 4):
        sel, sc, _ = engine.multikrum(X, f)
        osel, osc, _ = oracle.krum(X, f)
        assert np.array_equal(sel, osel)
        np.testing.assert_array_equal(np.isnan(sc), np.isnan(osc))
        fin = np.isfinite(osc)
        np.testing.assert_allclose(sc[fin], osc[fin], rtol=1e-12, atol=0)


def test_concurrent_callers_one_context_and_two(oracle):
    """The Go verifier calls from goroutines on arbitrary OS threads
    (krum.go:194,284 serialise Krum with krumLock, but the miner-side calls
    do not): 6 Python threads share one context, 2 more use a second context
    on the same device; every result must equal the oracle's."""
    import threading
    from biscotti_amd.krum import Engine
    cases = [(60 + 7 * i, 400 + 33 * i, 10 + i) for i in range(8)]
    data = [oracle.synth(n, d, 500 + i, f) for i, (n, d, f) in enumerate(cases)]
    want = [oracle.krum(X, f) for X, (n, d, f) in zip(data, cases)]
    e1, e2 = Engine(0), Engine(0)
    errors = []

    def run(i, eng):
        try:
            for _ in range(3):
                sel, sc, mean = eng.multikrum(data[i], cases[i][2])
                assert np.array_equal(sel, want[i][0])
                scale = float(np.max(np.mean(np.abs(data[i][want[i][0]]), axis=0)))
                assert float(np.max(np.abs(mean - want[i][2]))) <= 1e-9 * scale
        except Exception as ex:  # surfaced below
            errors.append((i, repr(ex)))

    ts = [threading.Thread(target=run, args=(i, e1 if i < 6 else e2)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    e1.close()
    e2.close()
    assert not errors, errors


def _split_engine(monkeypatch, parts, fail=0):
    """A 1-rank RCCL communicator that scores in `parts` row shares, as that
    many ranks would (BK_TEST_SPLIT_SCORES; read at bk_create)."""
    from biscotti_amd.krum import Engine, comm_unique_id
    monkeypatch.setenv("BK_TEST_SPLIT_SCORES", str(parts))
    if fail:
        monkeypatch.setenv("BK_TEST_SPLIT_FAIL", str(fail))
    e = Engine(0)
    monkeypatch.delenv("BK_TEST_SPLIT_SCORES")
    monkeypatch.delenv("BK_TEST_SPLIT_FAIL", raising=False)
    e.set_stream(torch.cuda.current_stream().cuda_stream)
    e.comm_init(1, 0, comm_unique_id())
    return e


@pytest.mark.parametrize("parts", [2, 3, 8])
@pytest.mark.parametrize("own_scores", [False, True])
def test_split_scores_bitwise(engine, monkeypatch, parts, own_scores):
    """Split scoring (n >= 2049 on the sharded entry: each rank scores its
    ceil(n / R) rows, one all-gather hands every rank all n scores): the R
    shares computed as R ranks would, on one GPU, give the unsplit call's
    selection, scores, mean and margin record bitwise -- with the caller's
    scores array or without one (libbk's own)."""
    e2 = _split_engine(monkeypatch, parts)
    try:
        n, d, f = 2100, 3000, 630
        X = torch.empty((n, d), dtype=torch.float64, device="cuda")
        engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 17, f)
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        sc = torch.empty(n, dtype=torch.float64, device="cuda")
        mean = torch.empty(d, dtype=torch.float64, device="cuda")
        e2.timing_enable(True)
        for _ in range(2):
            e2.multikrum_sharded_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(),
                                     None if own_scores else sc.data_ptr(), mean.data_ptr())
        e2.synchronize()
        t = e2.timing_read()
        e2.timing_enable(False)
        assert t["k_scores"]["count"] == 2 * parts  # one launch per share
        fsel, fsc, fmean = _dev_run(engine, X, f)
        assert np.array_equal(sel.cpu().numpy(), fsel)
        if not own_scores:
            assert np.array_equal(sc.cpu().numpy().view(np.int64), fsc.view(np.int64))
        assert np.array_equal(mean.cpu().numpy().view(np.int64), fmean.view(np.int64))
        m2, m1 = e2.selection_margin(), engine.selection_margin()
        assert m2 == m1
    finally:
        e2.close()


@pytest.mark.parametrize("form", ["f64_deterministic", "f32_i8x2_certified", "f32_mfma"])
def test_split_scores_other_forms(engine, monkeypatch, form):
    """Split scoring under the deterministic exchange (all-gather + rank-order
    sum) and on fp32 rows in the modes config E runs at 8 GPUs (the certified
    two-digit int8 Gram, the fp32 MFMA): 8 shares give the unsplit call's
    selection, scores and mean bitwise."""
    e2 = _split_engine(monkeypatch, 8)
    try:
        n, d, f = 2200, 2048, 660
        f32 = form.startswith("f32")
        dt = _lib.BK_F32 if f32 else _lib.BK_F64
        X = torch.empty((n, d), dtype=torch.float32 if f32 else torch.float64, device="cuda")
        engine.synth_fill_ptr(X.data_ptr(), dt, n, d, d, 0, d, 29, f)
        mode = {"f32_i8x2_certified": _lib.BK_F32_I8X2_CERTIFIED, "f32_mfma": _lib.BK_F32_MFMA}
        if form == "f64_deterministic":
            e2.comm_set_mode(True)
        outs = []
        for eng, sharded in ((e2, True), (engine, False)):
            if f32:
                eng.set_f32_mode(mode[form])
            sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
            sc = torch.empty(n, dtype=torch.float64, device="cuda")
            mean = torch.empty(d, dtype=torch.float64, device="cuda")
            try:
                call = eng.multikrum_sharded_ptr if sharded else eng.multikrum_device_ptr
                call(X.data_ptr(), dt, n, d, d, f, sel.data_ptr(), sc.data_ptr(), mean.data_ptr())
                eng.synchronize()
            finally:
                eng.set_f32_mode(_lib.BK_F32_EXACT)
            outs.append((sel.cpu().numpy(), sc.cpu().numpy(), mean.cpu().numpy()))
        (s1, c1, m1), (s2, c2, m2) = outs
        assert np.array_equal(s1, s2)
        assert np.array_equal(c1.view(np.int64), c2.view(np.int64))
        assert np.array_equal(m1.view(np.int64), m2.view(np.int64))
    finally:
        e2.close()


def test_split_scores_below_threshold_and_failed_share(engine, monkeypatch):
    """n = 2048 stays on one K2 launch (the split needs the transposed path);
    a share that fails on another rank marks the call invalid on this one
    (its NaN status word poisons the Gram record: BK_ERCCL, as a shard that
    fails before the exchange)."""
    e2 = _split_engine(monkeypatch, 4)
    try:
        n, d, f = 2048, 1000, 614
        X = torch.empty((n, d), dtype=torch.float64, device="cuda")
        engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 19, f)
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        e2.timing_enable(True)
        e2.multikrum_sharded_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr())
        e2.synchronize()
        assert e2.timing_read()["k_scores"]["count"] == 1
        e2.timing_enable(False)
        assert np.array_equal(sel.cpu().numpy(), _dev_run(engine, X, f)[0])
    finally:
        e2.close()
    e3 = _split_engine(monkeypatch, 3, fail=2)
    try:
        n, d, f = 2100, 1000, 630
        X = torch.empty((n, d), dtype=torch.float64, device="cuda")
        engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 23, f)
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        e3.multikrum_sharded_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr())
        with pytest.raises(_lib.BKError) as ei:
            e3.synchronize()
        assert ei.value.status == _lib.BK_ERCCL
    finally:
        e3.close()
