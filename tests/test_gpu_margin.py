"""The selection margin (include/bk.h bk_selection_margin) and the near-tie
contract on an MI355X.

The reference selects with np.argpartition over BLAS-rounded scores
(ML/code/logistic_validator.py:45, 59-63), so no rounding-different
implementation can promise its exact set unconditionally.  libbk reports, per
call, the boundary gap and a rigorous bound on how far any fp64 evaluation
(this one, numpy's) can sit from the exact scores: gap > err_bound proves the
reference selects the same set; otherwise the call is flagged near_tie.

* every small golden: the device record matches its definition (gap bitwise
  from the same call's scores, bound from the formula), and near_tie is set
  exactly on the goldens that are real ties (k = 0, all-zero rows);
* the tight goldens (boundary inside the honest cluster, relative gaps
  2.7e-8 .. 2.8e-12): the exact path matches bit-exactly, and its flag agrees
  with the bound evaluated on the golden (E_tight_fp32's boundary gap, 3.8e-6
  on scores of 1.4e6, is below the rigorous fp64 bound: flagged, yet matched);
* the fp32 MFMA path at its tolerance: it matches the golden or flags a near
  tie with gap <= err_bound -- never silently different -- and
  BK_F32_CERTIFIED always returns the golden set.
"""
import numpy as np
import pytest

import golden_util as GU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402


def _device_batch(engine, name):
    p = GU.C.case_params(name)
    n, d = p["n"], p["d"]
    tdt = torch.float32 if p["dtype"] == "float32" else torch.float64
    dt = _lib.BK_F32 if p["dtype"] == "float32" else _lib.BK_F64
    X = torch.empty((n, d), dtype=tdt, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), dt, n, d, X.stride(0), 0, d, p["seed"], p["nbyz"],
                          p["mu_scale"], p["byz_scale"], p["sigma"], p["flags"])
    return X, dt, p


def _run(engine, X, dt, f):
    n, d = X.shape
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mean = torch.empty(d, dtype=torch.float64, device="cuda")
    engine.multikrum_device_ptr(X.data_ptr(), dt, n, d, X.stride(0), f, sel.data_ptr(),
                                sc.data_ptr(), mean.data_ptr())
    engine.synchronize()
    return sel.cpu().numpy(), sc.cpu().numpy(), mean.cpu().numpy()


@pytest.mark.parametrize("name", GU.small_cases())
def test_margin_small_goldens(name, engine, oracle):
    X, p = GU.build_input(name, oracle)
    if p["error"]:
        pytest.skip("f = 0: the reference raises, no margin")
    n, d, f = p["n"], p["d"], p["f"]
    g = GU.load(name)
    sel, sc, _ = engine.multikrum(X, f)
    mg = engine.selection_margin()
    GU.check_margin(mg, sc, g["sq"], n, f, d)
    assert mg["near_tie"] == p["tie"], (name, mg)
    if not mg["near_tie"]:
        assert np.array_equal(sel, g["sel"])


@pytest.mark.parametrize("name", [k for k in ("C_tight", "E_tight_fp32", "D_512x1M_f256",
                                               "fp32_tight_700x65536") if GU.have(k)])
def test_tight_goldens_exact_path(name, engine):
    """Boundary inside the honest cluster: the exact path (fp64, or fp32 widened
    onto the fp64 MFMA) selects bit-exactly, and certifies exactly the goldens
    whose gap clears the bound (evaluated on the golden's own norms)."""
    X, dt, p = _device_batch(engine, name)
    n, d, f = p["n"], p["d"], p["f"]
    rec = GU.manifest()[name]
    sel, sc, mean = _run(engine, X, dt, f)
    g = GU.load(name)
    mg = engine.selection_margin()
    GU.check_margin(mg, sc, g["sq"], n, f, d)
    sq = g["sq"]
    want_bound = GU.margin_bound(float(np.max(sq[np.isfinite(sq)])), d, n - f - 2)
    if abs(rec["gap"] - want_bound) > 0.01 * want_bound:
        assert mg["near_tie"] == (not rec["gap"] > want_bound), (mg, rec["gap"], want_bound)
    assert np.array_equal(sel, g["sel"])
    GU.check_scores(sc, g, rel=1e-9)
    GU.check_mean(mean, g, rec)
    # the boundary really is tight: the relative gap is far below what the
    # r1 A-E goldens exercised (~1.0)
    assert rec["gap"] / rec["max_score"] < 1e-4
    del X
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", [k for k in ("fp32_tight_700x65536", "E_tight_fp32",
                                               "E_4096x262144_fp32", "fp32_200x3000")
                                  if GU.have(k)])
def test_f32_mfma_matches_or_flags(name, engine):
    """The fp32 MFMA path near its tolerance: the
    selection equals the golden, or the call is flagged near_tie with
    gap <= err_bound (never silently wrong); BK_F32_CERTIFIED re-runs exactly on
    a flag and always returns the golden set."""
    X, dt, p = _device_batch(engine, name)
    assert dt == _lib.BK_F32
    n, d, f = p["n"], p["d"], p["f"]
    g = GU.load(name)
    try:
        engine.set_f32_mode(_lib.BK_F32_MFMA)
        sel, sc, _ = _run(engine, X, dt, f)
        mg = engine.selection_margin()
        GU.check_margin(mg, sc, g["sq"], n, f, d, u_gram=2.0 ** -24)
        if not np.array_equal(sel, g["sel"]):
            assert mg["near_tie"] and not mg["gap"] > mg["err_bound"], mg
        flagged = mg["near_tie"]
        engine.set_f32_mode(_lib.BK_F32_CERTIFIED)
        r0 = engine.certified_reruns()
        sel2, sc2, mean2 = _run(engine, X, dt, f)
        assert np.array_equal(sel2, g["sel"])
        assert engine.certified_reruns() - r0 == (1 if flagged else 0)
        mg2 = engine.selection_margin()
        if flagged:  # the record is the exact re-run's
            GU.check_margin(mg2, sc2, g["sq"], n, f, d)
        GU.check_mean(mean2, g, GU.manifest()[name])
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
    del X
    torch.cuda.empty_cache()


def test_certified_host_entry(engine, oracle):
    """BK_F32_CERTIFIED through the host entry (bk_multikrum): the re-run reuses
    the staged device batch."""
    name = "fp32_tight_700x65536"
    if not GU.have(name):
        pytest.skip("golden not generated")
    X, p = GU.build_input(name, oracle)
    g = GU.load(name)
    try:
        engine.set_f32_mode(_lib.BK_F32_CERTIFIED)
        sel, sc, mean = engine.multikrum(X, p["f"])
        assert np.array_equal(sel, g["sel"])
        assert not engine.selection_margin()["near_tie"]
        GU.check_mean(mean, g, GU.manifest()[name])
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)


def test_margin_of_summed_shards_counts_all_columns(engine):
    """The packed partials' trailing records sum to the total d (and to 0 fp32-MFMA
    columns), so the margin after a multi-GPU exchange uses the whole batch's
    column count."""
    from biscotti_amd.dist import all_shards
    n, d, f = 200, 30011, 60
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 21, 40)
    usz = int(_lib.lib().bk_upper_elems(n))
    acc = torch.zeros(usz, dtype=torch.float64, device="cuda")
    for c0, dl in all_shards(d, 3):
        U = torch.empty(usz, dtype=torch.float64, device="cuda")
        engine.gram_upper_ptr(X[:, c0:].data_ptr(), _lib.BK_F64, n, dl, X.stride(0), U.data_ptr())
        engine.synchronize()
        assert float(U[-4]) == dl and float(U[-3]) == 0.0 and float(U[-2]) == 0.0
        acc += U
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    engine.finish_ptr(acc.data_ptr(), X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(),
                      sc.data_ptr(), None)
    engine.synchronize()
    mg = engine.selection_margin()
    assert mg["d"] == d
    s = sc.cpu().numpy()
    full = _run(engine, X, _lib.BK_F64, f)
    assert np.array_equal(sel.cpu().numpy(), full[0])
    mg_full = engine.selection_margin()
    assert mg_full["d"] == d and mg_full["k"] == mg["k"] == n - f - 2
    assert abs(mg["gap"] - mg_full["gap"]) <= 1e-9 * np.max(np.abs(s))


def test_empty_shard_joins_and_finishes(engine):
    """d_local = 0 (an empty trailing shard): the sharded entry accepts it,
    contributes a zero partial and still finishes."""
    n, f = 50, 10
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    engine.multikrum_sharded_ptr(None, _lib.BK_F64, n, 0, 0, f, sel.data_ptr(), sc.data_ptr(),
                                 None)
    engine.synchronize()
    assert np.array_equal(sel.cpu().numpy(), np.arange(n - f))  # all scores 0: lowest indices
    assert np.all(sc.cpu().numpy() == 0)
    mg = engine.selection_margin()
    assert mg["near_tie"] and mg["d"] == 0
    assert mg["err_bound"] == float("inf")  # no column count: the bound is unknown


def test_f32_mfma_record_carries_its_roundoff(engine, oracle):
    """the margin's unit roundoff travels in the packed record, so a
    finish on another context (a multi-GPU exchange) cannot under-estimate the
    bound: fp32-MFMA shards mark their columns, and one such shard in the sum
    makes the whole record u_G = 2^-24."""
    from biscotti_amd import dist as D
    from biscotti_amd.krum import Engine
    n, d, f = 300, 20000, 90
    X = torch.empty((n, d), dtype=torch.float32, device="cuda")
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, 0, d, 33, 60)
    usz = int(_lib.lib().bk_upper_elems(n))
    shards = D.all_shards(d, 2)
    other = Engine(0)  # an exact context for shard 1, the finish on a third view
    try:
        engine.set_f32_mode(_lib.BK_F32_MFMA)
        acc = torch.zeros(usz, dtype=torch.float64, device="cuda")
        for (c0, dl), eng in zip(shards, (engine, other)):
            U = torch.empty(usz, dtype=torch.float64, device="cuda")
            eng.gram_upper_ptr(X[:, c0:].data_ptr(), _lib.BK_F32, n, dl, X.stride(0), U.data_ptr())
            eng.synchronize()
            assert float(U[-4]) == dl
            assert float(U[-3]) == (dl if eng is engine else 0.0)
            acc += U
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        sc = torch.empty(n, dtype=torch.float64, device="cuda")
        other.finish_ptr(acc.data_ptr(), X.data_ptr(), _lib.BK_F32, n, d, d, f, sel.data_ptr(),
                         sc.data_ptr(), None)  # an exact context: the record decides
        other.synchronize()
        mg = other.selection_margin()
        sq = oracle.sqnorms(X.cpu().numpy())
        GU.check_margin(mg, sc.cpu().numpy(), sq, n, f, d, u_gram=2.0 ** -24)
        # a record without a column count: unknown bound, always a near tie
        acc[-4] = 0.0
        acc[-3] = 0.0
        other.finish_ptr(acc.data_ptr(), X.data_ptr(), _lib.BK_F32, n, d, d, f, sel.data_ptr(),
                         sc.data_ptr(), None)
        mg0 = other.selection_margin()
        assert mg0["near_tie"] and mg0["err_bound"] == float("inf")
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
        other.close()
