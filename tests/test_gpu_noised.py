"""MI355X parity of bk_multikrum_noised: the noise
application (DistSys/main.go:1524-1537, 1606-1653) fused into the H2D staging
of the verifier batch, then Multi-Krum (krum.go:100-166 ->
logistic_validator.py:36-65) on the noised rows.

Checked against the CPU oracle run in two steps on the same inputs:
oracle.noise (the noised batch, bit-exact) then oracle.krum (the selected set
bit-exact, the mean within the SURVEY §8(d) norm-wise 1e-9 bound).  The
column-chunk size (BK_STAGE_CHUNK_BYTES) is forced small so several chunks
cycle through the 2-slot noise ring and the chunk Gram partials are summed.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402


def _clustered(n, d, nbyz, seed):
    rng = np.random.default_rng(seed)
    mu = 0.01 * rng.standard_normal(d)
    X = mu + 1e-3 * rng.standard_normal((n, d))
    byz = rng.choice(n, nbyz, replace=False)
    X[byz] += 0.05 * rng.standard_normal((nbyz, d))
    return X


def _check(got, want_sel, want_mean, X):
    sel, _, mean, _ = got
    assert np.array_equal(np.sort(sel), np.sort(want_sel))
    scale = np.max(np.abs(X[want_sel]).sum(0) / len(want_sel))
    assert np.max(np.abs(mean - want_mean)) <= 1e-9 * scale


@pytest.mark.parametrize("n,d,k,f,chunk", [
    (10, 25, 2, 2, 0),          # config A shape
    (33, 1001, 3, 9, 4096),     # odd d (padded device rows), 64-column chunks, ragged last
    (100, 7850, 2, 30, 1 << 20),  # config B shape, 448-column chunks
    (64, 4096, 1, 19, 0),       # one chunk
    (20, 517, 0, 6, 0),         # k = 0: NoisedDelta = Delta
])
def test_noised_vs_oracle(engine, oracle, monkeypatch, n, d, k, f, chunk):
    if chunk:
        monkeypatch.setenv("BK_STAGE_CHUNK_BYTES", str(chunk))
    rng = np.random.default_rng(n * 31 + d + k)
    delta = _clustered(n, d, f // 2 + 1, n + d)
    noise = rng.standard_normal((n, k, d)) * 1e-4
    noised = oracle.noise(delta, noise) if k else delta.copy()
    want_sel, _, want_mean = oracle.krum(noised, f)
    got = engine.multikrum_noised(delta, noise, f, want_noised=True)
    assert np.array_equal(got[3].view(np.int64), noised.view(np.int64))
    _check(got, want_sel, want_mean, noised)


def test_noised_strided_pinned(engine, oracle):
    """row strides ld / noise_ld / out_ld > d and pinned host buffers through the
    pointer entry; the noised batch equals bk_noise_apply_device's bitwise."""
    n, d, k, f, ld = 48, 3000, 2, 14, 3003
    rng = np.random.default_rng(5)
    D = torch.empty((n, ld), dtype=torch.float64).pin_memory()
    D.copy_(torch.from_numpy(np.pad(_clustered(n, d, 7, 9), ((0, 0), (0, ld - d)))))
    N = torch.from_numpy(rng.standard_normal((n, k, ld)) * 1e-4).pin_memory()
    out = torch.zeros((n, ld), dtype=torch.float64).pin_memory()
    sel = torch.zeros(n - f, dtype=torch.int64)
    sc = torch.zeros(n, dtype=torch.float64)
    mean = torch.zeros(d, dtype=torch.float64)
    os.environ["BK_STAGE_CHUNK_BYTES"] = str(n * (1 + k) * 8 * 640)  # 640 columns: 5 chunks, ragged last
    try:
        m = engine.multikrum_noised_ptr(D.data_ptr(), ld, N.data_ptr(), k, ld,
                                        _lib.BK_HOST_PINNED, n, d, f, sel.data_ptr(),
                                        sc.data_ptr(), mean.data_ptr(), out.data_ptr(), ld)
    finally:
        del os.environ["BK_STAGE_CHUNK_BYTES"]
    assert m == n - f
    Dn, Nn = D.numpy()[:, :d], N.numpy()[:, :, :d]
    noised = oracle.noise(Dn, Nn)
    assert np.array_equal(out.numpy()[:, :d].view(np.int64), noised.view(np.int64))
    # the device kernel alone gives the same bits
    tD, tN = D.cuda(), N.cuda()
    o2 = torch.empty((n, ld), dtype=torch.float64, device="cuda")
    engine.noise_apply_ptr(tD.data_ptr(), n, d, ld, tN.data_ptr(), k, ld, o2.data_ptr(), ld)
    engine.synchronize()
    assert np.array_equal(o2.cpu().numpy()[:, :d].view(np.int64), noised.view(np.int64))
    want_sel, want_sc, want_mean = oracle.krum(noised, f)
    _check((sel.numpy(), None, mean.numpy(), None), want_sel, want_mean, noised)
    assert np.max(np.abs(sc.numpy() - want_sc)) <= 1e-9 * np.max(np.abs(want_sc))


def test_noised_repeated_calls_and_errors(engine, oracle):
    """back-to-back calls reuse the ring and batch buffers; argument errors are
    reported, never aborted."""
    n, d, k, f = 40, 2048, 3, 12
    rng = np.random.default_rng(11)
    os.environ["BK_STAGE_CHUNK_BYTES"] = str(n * (1 + k) * 8 * 256)
    try:
        for it in range(3):
            delta = _clustered(n, d, 6, 100 + it)
            noise = rng.standard_normal((n, k, d)) * 1e-4
            noised = oracle.noise(delta, noise)
            want_sel, _, want_mean = oracle.krum(noised, f)
            _check(engine.multikrum_noised(delta, noise, f), want_sel, want_mean, noised)
    finally:
        del os.environ["BK_STAGE_CHUNK_BYTES"]
    delta = np.zeros((4, 8))
    with pytest.raises(Exception):
        engine.multikrum_noised(delta, np.zeros((4, 1, 8)), 0)  # f = 0: the ValueError case
    with pytest.raises(Exception):
        engine.multikrum_noised_ptr(delta.ctypes.data, 8, None, 1, 8, _lib.BK_HOST, 4, 8, 1,
                                    np.zeros(3, np.int64).ctypes.data)  # k > 0, null noise
    with pytest.raises(Exception):
        engine.multikrum_noised_ptr(delta.ctypes.data, 8, None, 0, 8, _lib.BK_DEVICE, 4, 8, 1,
                                    np.zeros(3, np.int64).ctypes.data)  # device batches: EINVAL


@pytest.mark.parametrize("n,d,f,dtype,chunk_cols", [
    (512, 65536, 153, "f64", 4096),   # 16 chunks
    (100, 7850, 30, "f64", 1024),     # ragged last chunk
    (64, 9001, 19, "f64", 64),        # odd d, 47 chunks (the 64-chunk cap)
    (96, 20000, 28, "f32", 2048),     # fp32 rows
])
def test_host_entry_chunked_vs_device(engine, oracle, monkeypatch, n, d, f, dtype, chunk_cols):
    """bk_multikrum from host memory runs the column-chunked pipeline (copies
    overlapped with per-chunk K1): selection = oracle, mean bitwise = the
    device-resident entry (K4 reads the same rows), scores within 1e-9."""
    es = 4 if dtype == "f32" else 8
    monkeypatch.setenv("BK_STAGE_CHUNK_BYTES", str(n * es * chunk_cols))
    X = _clustered(n, d, f // 2 + 1, n * 3 + d)
    if dtype == "f32":
        X = X.astype(np.float32)
    sel, sc, mean = engine.multikrum(X, f)
    want_sel, want_sc, want_mean = oracle.krum(X, f)
    assert np.array_equal(sel, want_sel)
    X64 = X.astype(np.float64)
    scale = np.max(np.abs(X64[want_sel]).sum(0) / len(want_sel))
    assert np.max(np.abs(mean - want_mean)) <= 1e-9 * scale
    assert np.max(np.abs(sc - want_sc)) <= 1e-9 * np.max(np.abs(want_sc))
    tX = torch.from_numpy(X).cuda()
    dsel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    dmean = torch.empty(d, dtype=torch.float64, device="cuda")
    dt = _lib.BK_F32 if dtype == "f32" else _lib.BK_F64
    engine.multikrum_device_ptr(tX.data_ptr(), dt, n, d, d, f, dsel.data_ptr(), None,
                                dmean.data_ptr())
    engine.synchronize()
    assert np.array_equal(dsel.cpu().numpy(), sel)
    assert np.array_equal(dmean.cpu().numpy().view(np.int64), mean.view(np.int64))
