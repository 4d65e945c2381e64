"""MI355X: fp32 rows on the fp32 MFMA (bk_set_f32_mode(ctx, BK_F32_MFMA); BASELINE
config E's "fp32 MFMA path", SURVEY.md §8(d) tolerance re-stated).

* Fragment-layout check with exact data: small-integer fp32 rows make every
  product and partial sum exact in fp32, so the fp32-MFMA Gram must equal the
  exact (fp64-MFMA) one bit for bit -- over ragged n and d, the balanced band
  quads (n = 512) and the many-group plan (n = 1000).
* Config E at full size (4096 x 262144) against its golden: selection equal
  (the golden's boundary gap, 1.08e6, is far above the fp32 Gram error
  bound), scores within the re-stated bound
  2 k gamma_d max|x_i|^2 with gamma_d = d 2^-24, mean within 1e-9 (K4 is
  unchanged: fp64 accumulation of the fp32 rows).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402
import golden_util as GU  # noqa: E402


@pytest.fixture
def f32eng(engine):
    engine.set_f32_mode(_lib.BK_F32_MFMA)
    yield engine
    engine.set_f32_mode(_lib.BK_F32_EXACT)


def _upper(engine, X):
    n, d = X.shape
    tX = torch.from_numpy(np.ascontiguousarray(X)).cuda()
    U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
    engine.gram_upper_ptr(tX.data_ptr(), _lib.BK_F32, n, d, d, U.data_ptr())
    engine.synchronize()
    return U.cpu().numpy()


@pytest.mark.parametrize("n,d", [(64, 32), (100, 3001), (200, 4096), (512, 4000), (1000, 2048),
                                 (130, 37)])
def test_layout_exact_on_small_integers(engine, n, d):
    rng = np.random.default_rng(n + d)
    X = rng.integers(-8, 9, size=(n, d)).astype(np.float32)
    engine.set_f32_mode(_lib.BK_F32_EXACT)
    want = _upper(engine, X)
    engine.set_f32_mode(_lib.BK_F32_MFMA)
    try:
        got = _upper(engine, X)
    finally:
        engine.set_f32_mode(_lib.BK_F32_EXACT)
    assert np.array_equal(got[:-4], want[:-4])  # the tiles, bit for bit
    # the trailing record: the column count, and the columns taken on the fp32
    # MFMA (the K1 v3 kernel, 16-B aligned rows; v1 has no fp32 MFMA)
    assert got[-4] == want[-4] == d and want[-3] == 0.0
    assert got[-3] == (d if d % 4 == 0 else 0.0)
    assert got[-2] == want[-2] == 0.0 and got[-1] == want[-1] == 0.0


def test_clustered_vs_oracle(f32eng, oracle):
    n, d, f = 300, 20000, 90
    rng = np.random.default_rng(3)
    mu = 0.01 * rng.standard_normal(d)
    X = (mu + 1e-3 * rng.standard_normal((n, d))).astype(np.float32)
    byz = rng.choice(n, f, replace=False)
    X[byz] += (0.05 * rng.standard_normal((f, d))).astype(np.float32)
    sel, sc, mean = f32eng.multikrum(X, f)
    osel, osc, omean = oracle.krum(X, f)
    assert np.array_equal(sel, osel)
    k = n - f - 2
    X64 = X.astype(np.float64)
    bound = 2 * k * (d * 2.0 ** -24) * np.max(np.einsum("ij,ij->i", X64, X64))
    assert np.max(np.abs(sc - osc)) <= bound
    scale = np.max(np.abs(X64[osel]).sum(0) / len(osel))
    assert np.max(np.abs(mean - omean)) <= 1e-9 * scale


@pytest.mark.parametrize("name", [c for c in GU.large_cases() if "fp32" in c])
def test_config_E_golden(f32eng, name):
    p = GU.C.case_params(name)
    n, d, f = p["n"], p["d"], p["f"]
    X = torch.empty((n, d), dtype=torch.float32, device="cuda")
    f32eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, 0, d, p["seed"], p["nbyz"],
                          p["mu_scale"], p["byz_scale"], p["sigma"], p["flags"])
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mean = torch.empty(d, dtype=torch.float64, device="cuda")
    f32eng.multikrum_device_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, f, sel.data_ptr(),
                                sc.data_ptr(), mean.data_ptr())
    f32eng.synchronize()
    g = GU.load(name)
    # the separated config-E golden selects identically; the tight ones (boundary
    # inside the honest cluster) may differ, but only with the near-tie flag
    # raised (tests/test_gpu_margin.py checks the record itself)
    same = np.array_equal(sel.cpu().numpy(), g["sel"])
    if not same:
        mg = f32eng.selection_margin()
        assert mg["near_tie"] and not mg["gap"] > mg["err_bound"], mg
    if name == "E_4096x262144_fp32":
        assert np.array_equal(sel.cpu().numpy(), g["sel"])
    k = n - f - 2
    bound = 2 * k * (d * 2.0 ** -24) * float(np.max(g["sq"]))
    err = float(np.max(np.abs(sc.cpu().numpy() - g["scores"])))
    print("config E fp32 MFMA: max score error %.3e (bound %.3e, max score %.3e)"
          % (err, bound, float(np.max(g["scores"]))))
    assert err <= bound
    if same:  # a different (flagged) set has a different mean
        GU.check_mean(mean.cpu().numpy(), g, GU.manifest()[name])
    del X
    torch.cuda.empty_cache()
