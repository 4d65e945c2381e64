"""MI355X: K1i8, the Gram of fp32 rows from exact int8 digit slices
(bk_set_f32_mode(ctx, BK_F32_I8); bk_i8.hip; BASELINE config E, VERDICT r3
item 4).  The reference's Gram is np.dot(X, X.T) in fp64
(ML/code/logistic_validator.py:59-60).

* Layout and exactness: rows whose values are small integers times a per-row
  power of two are represented exactly by the digits, so the int8 Gram must
  equal the exact fp64 one BIT FOR BIT (ragged n and d, one to eight column
  ranges, the diagonal 128-row tiles and the padding).
* The absolute error bound: on random rows every element of the int8 Gram lies
  within the record's bound (its trailing element [2], recomputed here from
  the definition) of the exact Gram.
* Multi-Krum: every fp32 golden (config E at full size, its tight variant, the
  700 x 65,536 tight case): the selection equals the reference's, or the call is
  flagged near_tie with gap <= err_bound; BK_F32_I8_CERTIFIED always returns
  the reference's set.  The margin record matches its definition with the int8
  term.
* Non-finite input: the bound is +inf (always a near tie).
"""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402
import golden_util as GU  # noqa: E402


# the int8 modes: three digits (six products) and two digits (three products)
NS_OF = {_lib.BK_F32_I8: 3, _lib.BK_F32_I8_CERTIFIED: 3, _lib.BK_F32_I8X2: 2,
         _lib.BK_F32_I8X2_CERTIFIED: 2}
I8_MODES = [_lib.BK_F32_I8, _lib.BK_F32_I8X2]
CERT_OF = {_lib.BK_F32_I8: _lib.BK_F32_I8_CERTIFIED, _lib.BK_F32_I8X2: _lib.BK_F32_I8X2_CERTIFIED}
F64_OF = {_lib.BK_F32_I8: _lib.BK_F64_I8, _lib.BK_F32_I8X2: _lib.BK_F64_I8X2}
MODE_IDS = {_lib.BK_F32_I8: "3digit", _lib.BK_F32_I8X2: "2digit"}


def _upper(engine, X, mode):
    n, d = X.shape
    tX = torch.from_numpy(np.ascontiguousarray(X)).cuda()
    U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
    engine.set_f32_mode(mode)
    try:
        engine.gram_upper_ptr(tX.data_ptr(), _lib.BK_F32, n, d, d, U.data_ptr())
        engine.synchronize()
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
    return U.cpu().numpy()


def _ntiles(n, ns):
    """i8_layout's output tiles: 128-row blocks I against column blocks J of
    128 (three digits) or 256 (two digits) holding some of the upper triangle."""
    tj = 256 if ns == 2 else 128
    TI, TJ, rj = -(-n // 128), -(-n // tj), tj // 128
    return sum(1 for i in range(TI) for j in range(TJ) if i <= rj * j + rj - 1)


def _ranges(n, d, es, num_cu=256, ns=3):
    """bk_i8.hip i8_layout: R column ranges of whole 64-column granules, each
    row slice <= 128 KiB.  Rows that need fewer than 8 such ranges (a shard of
    a d-sharded call): R in [R0, 8] minimising workgroup rounds x (columns per
    range + 2048) + 3072 (n / 4096)^2 R.  Otherwise at least 8, in eights;
    then raised (in eights, up to 4x, ranges >= 16 chunks) when that fills the
    XCDs' last round of (tile, range) workgroups by more than 5 points."""
    dp = (d + 63) // 64 * 64
    nk = dp // 64
    cmax = 131072 // es
    R0 = -(-dp // cmax)
    NT = _ntiles(n, ns)
    if R0 < 8:
        c1 = 3072.0 * (n / 4096.0) * (n / 4096.0)

        def cost(r):
            return math.ceil(NT * r / num_cu) * (dp / r + 2048.0) + c1 * r
        R = R0
        for r in range(R0 + 1, min(8, nk) + 1):
            if cost(r) < cost(R):
                R = r
        return [(nk * r // R * 64, nk * (r + 1) // R * 64) for r in range(R)]
    R = -(-R0 // 8) * 8
    R = min(nk, R)
    cx = num_cu / 8.0

    def eff(r):
        rounds = (-(-(NT * r) // 8)) / cx
        return rounds / math.ceil(rounds)
    best, r = R, R + 8
    while r <= 4 * R and nk // r >= 16:
        if eff(r) > eff(best) + 0.05:
            best = r
        r += 8
    R = best
    return [(nk * r // R * 64, nk * (r + 1) // R * 64) for r in range(R)]


def _bound(X, ns=3):
    """bk_i8.hip's absolute bound, restated from its definition: per range
    2^-21 (2 S L1 + 2.03 d S^2) with three digits, 2^-14 (2 S L1 + 1.0001 d S^2)
    with two (the dropped a1 b1 2^-26 product and the remainders |rho| <= 2^-14)."""
    es = X.dtype.itemsize
    X = X.astype(np.float64)
    tot = 0.0
    for c0, c1 in _ranges(X.shape[0], X.shape[1], es, ns=ns):
        A = np.abs(X[:, c0:min(c1, X.shape[1])])
        if A.shape[1] == 0:
            continue
        mx = A.max(1)
        s = np.where(mx > 0, 2.0 ** np.where(mx > 0, np.frexp(mx)[1], 0), 1.0)
        S, L1 = float(s.max()), float(A.sum(1).max())
        if ns == 3:
            tot += 2.0 ** -21 * (2.0 * S * L1 + 2.03 * A.shape[1] * S * S)
        else:
            tot += 2.0 ** -14 * (2.0 * S * L1 + 1.0001 * A.shape[1] * S * S)
    return tot * (1.0 + 2.0 ** -20)


@pytest.mark.parametrize("n,d", [(129, 64), (130, 4096), (256, 4160), (300, 20000), (512, 4000),
                                 (1000, 780), (200, 70000), (520, 9000)])
@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_exact_on_scaled_small_integers(engine, n, d, mode):
    """Rows of small integers times a per-row power of two: three digits hold
    |k| <= 64 exactly, two digits (a1 = 0) |k| <= 63, so the int8 Gram is the
    exact one bit for bit."""
    ns = NS_OF[mode]
    rng = np.random.default_rng(n + d)
    X = rng.integers(-64, 65, size=(n, d)) if ns == 3 else rng.integers(-63, 64, size=(n, d))
    X = X.astype(np.float32)
    X *= (2.0 ** rng.integers(-10, 11, size=(n, 1))).astype(np.float32)  # per-row scales
    X[3] = 0.0  # an all-zero row
    from biscotti_amd.dist import unpack_upper
    want = _upper(engine, X, _lib.BK_F32_EXACT)
    got = _upper(engine, X, mode)
    # the Gram, bit for bit (a diagonal sub-tile's lower half is not part of
    # the packed contract: K1 leaves it, K1i8 writes it symmetric)
    assert np.array_equal(unpack_upper(got, n), unpack_upper(want, n))
    assert got[-4] == d and got[-3] == 0.0 and got[-1] == 0.0
    assert got[-2] == pytest.approx(_bound(X, ns), rel=1e-12)


@pytest.mark.parametrize("n,d,scale", [(257, 3000, 1.0), (640, 65536, 1e-3), (1024, 20000, 1e4),
                                       (150, 100000, 1.0), (700, 33000, 1.0)])
@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_error_within_the_bound(engine, n, d, scale, mode):
    from biscotti_amd.dist import unpack_upper
    ns = NS_OF[mode]
    rng = np.random.default_rng(d)
    X = (scale * rng.standard_normal((n, d))).astype(np.float32)
    X[: n // 4] *= np.float32(1e-3)  # rows of very different magnitude
    want = unpack_upper(_upper(engine, X, _lib.BK_F32_EXACT), n)
    U = _upper(engine, X, mode)
    got = unpack_upper(U, n)
    E = float(U[-2])
    assert E == pytest.approx(_bound(X, ns), rel=1e-12)
    err = float(np.max(np.abs(got - want)))
    print("K1i8 (%d digits) n=%d d=%d: max |G~ - G| %.3e, bound %.3e, max G_ii %.3e"
          % (ns, n, d, err, E, float(np.max(np.diag(want)))))
    assert err <= E
    assert np.array_equal(got, got.T)  # symmetric bit for bit


def _device_batch(engine, name):
    p = GU.C.case_params(name)
    n, d = p["n"], p["d"]
    X = torch.empty((n, d), dtype=torch.float32, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, 0, d, p["seed"], p["nbyz"],
                          p["mu_scale"], p["byz_scale"], p["sigma"], p["flags"])
    return X, p


def _run(engine, X, f):
    n, d = X.shape
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mean = torch.empty(d, dtype=torch.float64, device="cuda")
    engine.multikrum_device_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, f, sel.data_ptr(),
                                sc.data_ptr(), mean.data_ptr())
    engine.synchronize()
    return sel.cpu().numpy(), sc.cpu().numpy(), mean.cpu().numpy()


@pytest.mark.parametrize("name", [k for k in ("E_4096x262144_fp32", "E_tight_fp32",
                                               "fp32_tight_700x65536", "fp32_200x3000")
                                  if GU.have(k)])
@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_i8_matches_or_flags(name, engine, mode):
    X, p = _device_batch(engine, name)
    n, d, f = p["n"], p["d"], p["f"]
    g = GU.load(name)
    try:
        engine.set_f32_mode(mode)
        sel, sc, mean = _run(engine, X, f)
        mg = engine.selection_margin()
        assert mg["near_tie"] == (not (mg["gap"] > mg["err_bound"]))
        if not np.array_equal(sel, g["sel"]):
            assert mg["near_tie"] and not mg["gap"] > mg["err_bound"], mg
        else:
            GU.check_mean(mean, g, GU.manifest()[name])
        if name == "E_4096x262144_fp32":  # the config-E golden's gap clears the int8 bound
            assert not mg["near_tie"] and np.array_equal(sel, g["sel"])
        k = n - f - 2
        err = float(np.max(np.abs(sc - g["scores"])))
        print("%s K1i8 (%d digits): max score error %.3e, err_bound %.3e, gap %.3e, near_tie %s"
              % (name, NS_OF[mode], err, mg["err_bound"], mg["gap"], mg["near_tie"]))
        assert err <= mg["err_bound"] / 2 + 1e-9 * float(np.max(np.abs(g["scores"])))
        flagged = mg["near_tie"]
        engine.set_f32_mode(CERT_OF[mode])
        r0 = engine.certified_reruns()
        sel2, sc2, mean2 = _run(engine, X, f)
        assert np.array_equal(sel2, g["sel"])
        assert engine.certified_reruns() - r0 == (1 if flagged else 0)
        GU.check_mean(mean2, g, GU.manifest()[name])
        assert k == mg["k"]
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
    del X
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_i8_margin_record(engine, oracle, mode):
    """The device margin record of an int8 call against its definition: the
    gap from the call's own scores, the bound with the record's int8 term."""
    n, d, f = 300, 20000, 90
    rng = np.random.default_rng(3)
    mu = 0.01 * rng.standard_normal(d)
    X = (mu + 1e-3 * rng.standard_normal((n, d))).astype(np.float32)
    byz = rng.choice(n, f, replace=False)
    X[byz] += (0.05 * rng.standard_normal((f, d))).astype(np.float32)
    engine.set_f32_mode(mode)
    try:
        sel, sc, mean = engine.multikrum(X, f)
        mg = engine.selection_margin()
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
    osel, osc, omean = oracle.krum(X, f)
    assert np.array_equal(sel, osel) and not mg["near_tie"]
    GU.check_margin(mg, sc, oracle.sqnorms(X), n, f, d, eg=_bound(X, NS_OF[mode]))
    X64 = X.astype(np.float64)
    scale = np.max(np.abs(X64[osel]).sum(0) / len(osel))
    assert np.max(np.abs(mean - omean)) <= 1e-9 * scale


@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_unaligned_rows_take_the_exact_path(engine, mode):
    """K1i8 stages 16-B granules: rows with ld % 4 != 0 take the exact path
    (its record carries no int8 bound) and return the exact Gram."""
    from biscotti_amd.dist import unpack_upper
    rng = np.random.default_rng(4)
    X = rng.standard_normal((300, 777)).astype(np.float32)
    want = _upper(engine, X, _lib.BK_F32_EXACT)
    got = _upper(engine, X, mode)
    assert got[-2] == 0.0 and np.array_equal(unpack_upper(got, 300), unpack_upper(want, 300))


def test_i8_nonfinite_is_a_near_tie(engine):
    n, d, f = 200, 5000, 60
    rng = np.random.default_rng(9)
    X = rng.standard_normal((n, d)).astype(np.float32)
    X[17, 123] = np.inf
    U = _upper(engine, X, _lib.BK_F32_I8)
    assert U[-2] == np.inf
    engine.set_f32_mode(_lib.BK_F32_I8)
    try:
        engine.multikrum(X, f)
        assert engine.selection_margin()["near_tie"]
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)


@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_i8_nonfinite_rows_are_never_selected(engine, oracle, dtype, mode):
    """a row holding a NaN or an infinity must not look
    like the zero vector to the int8 Gram (its digits are zero).  Its Gram
    elements are NaN, so it scores NaN and ranks last -- as the reference's
    NaN / inf distances rank it (logistic_validator.py:59-63) -- and the
    selection equals the oracle's; the bound is +inf (near tie)."""
    from biscotti_amd.dist import unpack_upper
    n, d, f = 300, 9000, 90
    rng = np.random.default_rng(11)
    X = (0.01 * rng.standard_normal((n, d))).astype(dtype)
    X[17, 123] = np.inf   # one inf element
    X[40] = np.nan        # a whole NaN row
    X[41, 8999] = -np.inf  # in the last range
    X[5] = 0.0            # the all-zero row a NaN row used to look like
    mode_set = engine.set_f32_mode if dtype == np.float32 else engine.set_f64_mode
    i8 = mode if dtype == np.float32 else F64_OF[mode]
    tX = torch.from_numpy(X).cuda()
    U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
    mode_set(i8)
    try:
        engine.gram_upper_ptr(tX.data_ptr(), _lib.BK_F32 if dtype == np.float32 else _lib.BK_F64,
                              n, d, d, U.data_ptr())
        engine.synchronize()
        sel, sc, _ = engine.multikrum(X, f)
        mg = engine.selection_margin()
    finally:
        mode_set(0)
    G = unpack_upper(U.cpu().numpy(), n)
    for r in (17, 40, 41):
        assert np.all(np.isnan(G[r])) and np.all(np.isnan(G[:, r]))
    ok = np.setdiff1d(np.arange(n), [17, 40, 41])
    assert np.all(np.isfinite(G[np.ix_(ok, ok)]))
    assert mg["near_tie"]
    assert not {17, 40, 41} & set(sel.tolist())
    assert np.all(np.isnan(sc[[17, 40, 41]]))
    osel, osc, _ = oracle.krum(X, f)
    assert np.array_equal(sel, osel)


@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_i8_shard_records_sum(engine, mode):
    """Two column shards on the int8 path: each record carries its own bound,
    and the exchange's sum (here: on the host) finishes like the whole batch."""
    from biscotti_amd.dist import all_shards
    n, d, f = 400, 30000, 120
    rng = np.random.default_rng(5)
    X = (0.01 * rng.standard_normal((n, d))).astype(np.float32)
    tX = torch.from_numpy(X).cuda()
    usz = int(_lib.lib().bk_upper_elems(n))
    acc = torch.zeros(usz, dtype=torch.float64, device="cuda")
    bounds = []
    engine.set_f32_mode(mode)
    try:
        for c0, dl in all_shards(d, 2):
            U = torch.empty(usz, dtype=torch.float64, device="cuda")
            Xs = np.ascontiguousarray(X[:, c0:c0 + dl])
            tXs = torch.from_numpy(Xs).cuda()
            engine.gram_upper_ptr(tXs.data_ptr(), _lib.BK_F32, n, dl, dl, U.data_ptr())
            engine.synchronize()
            assert float(U[-4]) == dl and float(U[-2]) == pytest.approx(_bound(Xs, NS_OF[mode]), rel=1e-12)
            bounds.append(float(U[-2]))
            acc += U
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        sc = torch.empty(n, dtype=torch.float64, device="cuda")
        engine.finish_ptr(acc.data_ptr(), tX.data_ptr(), _lib.BK_F32, n, d, d, f, sel.data_ptr(),
                          sc.data_ptr(), None)
        engine.synchronize()
        mg = engine.selection_margin()
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
    assert mg["d"] == d
    want = GU.margin_bound(mg["M"], d, n - f - 2, eg=sum(bounds))
    assert abs(mg["err_bound"] - want) <= 1e-12 * want


@pytest.mark.parametrize("name", [k for k in ("C_1024x131072", "D_512x1M_f153", "C_tight", "B_tight",
                                               "n1000_d2000") if GU.have(k)])
@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_f64_i8_matches_or_flags(name, engine, oracle, mode):
    """fp64 rows on K1i8 (bk_set_f64_mode): the selection equals the
    reference's or is flagged; BK_F64_I8_CERTIFIED always returns the
    reference's set, and the mean (K4 on the fp64 rows) within the §8(d) bound."""
    p = GU.C.case_params(name)
    n, d, f = p["n"], p["d"], p["f"]
    if p["dtype"] != "float64":
        pytest.skip("fp64 cases only")
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, p["seed"], p["nbyz"],
                          p["mu_scale"], p["byz_scale"], p["sigma"], p["flags"])
    g = GU.load(name)
    dev_run = lambda: _run64(engine, X, f)
    try:
        engine.set_f64_mode(F64_OF[mode])
        sel, sc, mean = dev_run()
        mg = engine.selection_margin()
        if n > 128:  # n <= 128 takes k_small, always exact
            assert mg["err_bound"] > 0
        if not np.array_equal(sel, g["sel"]):
            assert mg["near_tie"] and not mg["gap"] > mg["err_bound"], mg
        err = float(np.max(np.abs(sc - g["scores"])))
        print("%s fp64 K1i8 (%d digits): max score error %.3e, err_bound %.3e, gap %.3e, near_tie %s"
              % (name, NS_OF[mode], err, mg["err_bound"], mg["gap"], mg["near_tie"]))
        assert err <= mg["err_bound"] / 2 + 1e-9 * float(np.max(np.abs(g["scores"])))
        engine.set_f64_mode(F64_OF[mode] + 1)  # its certified form
        sel2, _, mean2 = dev_run()
        assert np.array_equal(sel2, g["sel"])
        GU.check_mean(mean2, g, GU.manifest()[name])
    finally:
        engine.set_f64_mode(_lib.BK_F64_EXACT)
    del X
    torch.cuda.empty_cache()


def _run64(engine, X, f):
    n, d = X.shape
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mean = torch.empty(d, dtype=torch.float64, device="cuda")
    engine.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(),
                                sc.data_ptr(), mean.data_ptr())
    engine.synchronize()
    return sel.cpu().numpy(), sc.cpu().numpy(), mean.cpu().numpy()


@pytest.mark.parametrize("n,d", [(130, 4096), (300, 20000), (512, 70000)])
@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_f64_i8_error_within_the_bound(engine, n, d, mode):
    from biscotti_amd.dist import unpack_upper
    rng = np.random.default_rng(d + 1)
    X = rng.standard_normal((n, d))
    X[: n // 3] *= 1e-4
    tX = torch.from_numpy(X).cuda()
    usz = int(_lib.lib().bk_upper_elems(n))
    out = {}
    m64 = F64_OF[mode]
    for mode in (_lib.BK_F64_EXACT, m64):
        U = torch.empty(usz, dtype=torch.float64, device="cuda")
        engine.set_f64_mode(mode)
        try:
            engine.gram_upper_ptr(tX.data_ptr(), _lib.BK_F64, n, d, d, U.data_ptr())
            engine.synchronize()
        finally:
            engine.set_f64_mode(_lib.BK_F64_EXACT)
        out[mode] = U.cpu().numpy()
    E = float(out[m64][-2])
    assert E == pytest.approx(_bound(X, 3 if m64 == _lib.BK_F64_I8 else 2), rel=1e-12)
    err = float(np.max(np.abs(unpack_upper(out[m64], n) - unpack_upper(out[_lib.BK_F64_EXACT], n))))
    print("fp64 K1i8 n=%d d=%d: max err %.3e bound %.3e" % (n, d, err, E))
    assert err <= E


def test_i8_workspace_failure_runs_exact(oracle, monkeypatch):
    """when K1i8's workspace (R range partials of the packed upper)
    cannot be allocated the call runs on the exact path instead of failing
    with BK_ENOMEM (test knob BK_TEST_I8_ENOMEM, read at bk_create)."""
    from biscotti_amd.dist import unpack_upper
    from biscotti_amd.krum import Engine
    monkeypatch.setenv("BK_TEST_I8_ENOMEM", "1")
    eng = Engine(0)
    monkeypatch.delenv("BK_TEST_I8_ENOMEM")
    try:
        rng = np.random.default_rng(12)
        X = rng.standard_normal((300, 4000)).astype(np.float32)
        got = _upper(eng, X, _lib.BK_F32_I8)
        want = _upper(eng, X, _lib.BK_F32_EXACT)
        assert got[-2] == 0.0  # no int8 bound: the exact path ran
        assert np.array_equal(unpack_upper(got, 300), unpack_upper(want, 300))
        eng.set_f32_mode(_lib.BK_F32_I8)
        sel, _, _ = eng.multikrum(X, 90)
        eng.set_f32_mode(_lib.BK_F32_EXACT)
        assert np.array_equal(sel, oracle.krum(X, 90)[0])
    finally:
        eng.close()


@pytest.mark.parametrize("mode", I8_MODES, ids=MODE_IDS.get)
def test_i8_at_max_n(engine, oracle, mode):
    """BK_MAX_N = 16,384 rows on K1i8 (128 row blocks; two digits: 64 column
    blocks of 256, rows padded to 256): the Gram of digit-representable rows
    equals the exact one bit for bit, and Multi-Krum on them selects the
    oracle's set."""
    from biscotti_amd.dist import unpack_upper
    n, d, f = 16384, 192, 4915
    rng = np.random.default_rng(16384)
    X = rng.integers(-63, 64, size=(n, d)).astype(np.float32)
    X *= (2.0 ** rng.integers(-6, 7, size=(n, 1))).astype(np.float32)
    want = _upper(engine, X, _lib.BK_F32_EXACT)
    got = _upper(engine, X, mode)
    assert got[-2] == pytest.approx(_bound(X, NS_OF[mode]), rel=1e-12)
    Gw, Gg = unpack_upper(want, n), unpack_upper(got, n)
    assert np.array_equal(Gg, Gw)
    del Gw, Gg
    engine.set_f32_mode(mode)
    try:
        sel, _, _ = engine.multikrum(X, f)
        mg = engine.selection_margin()
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
    osel, _, _ = oracle.krum(X, f)
    assert np.array_equal(sel, osel) or mg["near_tie"]
