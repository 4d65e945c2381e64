"""The row-fed host entry bk_multikrum_rows: n separately
allocated host rows, as the Go verifier holds them (getTopKRUMIndex(deltas
[][]float64), DistSys/krum.go:100-166), packed by libbk's host threads into a
pinned ring while the chunks cross PCIe.

The bar: every output (selection, scores, mean) bitwise that of
bk_multikrum(BK_HOST_PINNED) on the same rows packed row-major into one pinned
batch -- the shim's old serial pack -- and the selection equal to the
reference golden; whatever the thread count, the chunking (forced down to
many chunks so the ring's slots are reused) and the rows' alignment."""
import ctypes
import os

import numpy as np
import pytest

import golden_util as GU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402


def _rows(X, offset=0):
    """n separate allocations holding X's rows; offset (elements) shifts each
    row inside a larger buffer (rows not 16-B aligned)."""
    out, keep = [], []
    for i in range(X.shape[0]):
        buf = np.empty(X.shape[1] + offset, dtype=X.dtype)
        buf[offset:] = X[i]
        keep.append(buf)
        out.append(buf[offset:])
    return out, keep


def _pinned(engine, X, f):
    n, d = X.shape
    Xh = torch.from_numpy(np.ascontiguousarray(X)).pin_memory()
    sel, sc, mean = np.empty(n - f, np.int64), np.empty(n), np.empty(d)
    mo = ctypes.c_int64(0)
    dt = _lib.BK_F32 if X.dtype == np.float32 else _lib.BK_F64
    _lib.check(_lib.lib().bk_multikrum(engine.ctx, ctypes.c_void_p(Xh.data_ptr()),
                                       _lib.BK_HOST_PINNED, dt, n, d, d, f, sel.ctypes.data,
                                       ctypes.addressof(mo), sc.ctypes.data, mean.ctypes.data))
    return sel, sc, mean


def _same(a, b):
    return (np.array_equal(a[0], b[0]) and
            np.array_equal(a[1].view(np.int64), b[1].view(np.int64)) and
            np.array_equal(a[2].view(np.int64), b[2].view(np.int64)))


@pytest.fixture
def chunk_env():
    """set BK_STAGE_CHUNK_BYTES for the duration of a test (read per call)"""
    old = os.environ.get("BK_STAGE_CHUNK_BYTES")

    def set_(v):
        os.environ["BK_STAGE_CHUNK_BYTES"] = str(v)
    yield set_
    if old is None:
        os.environ.pop("BK_STAGE_CHUNK_BYTES", None)
    else:
        os.environ["BK_STAGE_CHUNK_BYTES"] = old


@pytest.mark.parametrize("name", GU.small_cases())
def test_small_goldens_from_rows(name, engine, oracle):
    X, p = GU.build_input(name, oracle)
    if p["error"]:
        rows, _ = _rows(np.ascontiguousarray(X))
        with pytest.raises(ValueError):
            engine.multikrum_rows(rows, p["f"])
        return
    Xc = np.ascontiguousarray(X)
    rows, _ = _rows(Xc)
    got = engine.multikrum_rows(rows, p["f"])
    g = GU.load(name)
    assert np.array_equal(got[0], g["sel"]), name
    assert _same(got, _pinned(engine, Xc, p["f"])), name


@pytest.mark.parametrize("n,d,f,dtype", [
    (10, 25, 2, np.float64),        # config A's shape: k_tiny reads the pinned stage
    (100, 7850, 30, np.float64),    # config B's shape: row groups + k_small
    (128, 32768, 40, np.float32),   # the largest k_small shape, fp32
    (300, 40000, 90, np.float64),   # general path, one chunk
    (513, 4099, 153, np.float64),   # n not a multiple of 64
    (257, 2049, 77, np.float32)])
@pytest.mark.parametrize("threads", [1, 3, 16])
def test_rows_bitwise_pinned(engine, oracle, n, d, f, dtype, threads):
    X = oracle.synth(n, d, 4000 + n + d, f, dtype=dtype)
    rows, _ = _rows(X)
    engine.set_host_threads(threads)
    try:
        got = engine.multikrum_rows(rows, f)
    finally:
        engine.set_host_threads(0)
    assert _same(got, _pinned(engine, X, f))
    osel, _, _ = oracle.krum(X, f)
    assert np.array_equal(got[0], osel)


@pytest.mark.parametrize("chunk_bytes", [1 << 20, 3 << 20, 40 << 20])
def test_rows_many_chunks_ring_reuse(engine, oracle, chunk_env, chunk_bytes):
    """column chunks forced small: up to 64 chunks through the 3-slot ring,
    each slot reused many times while the copy engine reads the others"""
    n, d, f = 200, 50000, 60
    X = oracle.synth(n, d, 77, f)
    chunk_env(chunk_bytes)
    rows, _ = _rows(X, offset=1)  # 8-B aligned rows (the stage's stores realign)
    for threads in (1, 5):
        engine.set_host_threads(threads)
        try:
            got = engine.multikrum_rows(rows, f)
        finally:
            engine.set_host_threads(0)
        assert _same(got, _pinned(engine, X, f)), (chunk_bytes, threads)


def test_rows_certified_modes(engine, oracle):
    """the certified int8 modes through the row-fed entry: the same outputs as
    the pinned entry in the same mode (an approximate Gram, re-run exact on a
    near tie)"""
    n, d, f = 300, 20000, 90
    X = oracle.synth(n, d, 99, f)
    rows, _ = _rows(X)
    for mode in (_lib.BK_F64_I8X2_CERTIFIED, _lib.BK_F64_I8_CERTIFIED):
        engine.set_f64_mode(mode)
        try:
            got = engine.multikrum_rows(rows, f)
            ref = _pinned(engine, X, f)
        finally:
            engine.set_f64_mode(_lib.BK_F64_EXACT)
        assert _same(got, ref), mode
        assert np.array_equal(got[0], oracle.krum(X, f)[0])


def test_rows_errors(engine):
    X = np.ones((5, 10))
    rows = [X[i].copy() for i in range(5)]
    ptrs = (ctypes.c_void_p * 5)(*[r.ctypes.data for r in rows])
    ptrs[3] = None
    sel = np.empty(3, np.int64)
    mo = ctypes.c_int64(0)
    L = _lib.lib()
    assert L.bk_multikrum_rows(engine.ctx, ptrs, _lib.BK_F64, 5, 10, 2, sel.ctypes.data,
                               ctypes.addressof(mo), None, None) == _lib.BK_EINVAL
    assert "null row 3" in _lib.last_error()
    assert L.bk_multikrum_rows(engine.ctx, None, _lib.BK_F64, 5, 10, 2, sel.ctypes.data,
                               ctypes.addressof(mo), None, None) == _lib.BK_EINVAL
    with pytest.raises(ValueError):  # f = 0: the reference's argpartition ValueError
        engine.multikrum_rows(rows, 0)
    assert L.bk_set_host_threads(engine.ctx, -1) == _lib.BK_EINVAL


def test_config_d_from_rows(engine):
    """BASELINE's headline batch (512 x 1,048,576 fp64) as 512 separate 8 MB
    host rows: the golden's selection, every output bitwise the pinned entry's"""
    p = GU.C.case_params("D_512x1M_f153")
    n, d, f = p["n"], p["d"], p["f"]
    Xd = torch.empty((n, d), dtype=torch.float64, device="cuda")
    engine.synth_fill_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, 0, d, p["seed"], p["nbyz"],
                          p["mu_scale"], p["byz_scale"], p["sigma"], p["flags"])
    Xh = Xd.cpu().numpy()
    del Xd
    torch.cuda.empty_cache()
    rows, _ = _rows(Xh)
    got = engine.multikrum_rows(rows, f)
    g = GU.load("D_512x1M_f153")
    assert np.array_equal(got[0], g["sel"])
    GU.check_mean(got[2], g, GU.manifest()["D_512x1M_f153"])
    assert _same(got, _pinned(engine, Xh, f))
