"""k_small (bk_small.hip): the whole Multi-Krum of an n <= 128 batch in ONE
launch -- Biscotti's deployed verifier shapes (config A creditcard n <= 10,
d = 25; config B mnist 100 x 7,850).  Checked on the MI355X:

* every golden with n <= 128 through the device entry: the selection equals
  the reference's (bit-exact) wherever the margin certifies it, scores within
  1e-9, mean within the §8(d) bound, and the margin record matches its
  definition;
* against the general six-launch chain on the same batch: same selection,
  the mean BITWISE (same ascending order of adds), scores within rounding;
* ragged shapes: n = 2..128, d from 1 to non-multiples of 8, fp32 rows;
* hundreds of back-to-back launches over alternating shapes (the queue
  counters reset themselves), run-to-run bitwise determinism, and no hand-off
  wait ever times out (bk_selection_margin would report BK_EHIP).
"""
import numpy as np
import pytest

import golden_util as GU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402


def _run(e, X, f, scores=True, mean=True):
    n, d = X.shape
    dt = _lib.BK_F32 if X.dtype == torch.float32 else _lib.BK_F64
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda") if scores else None
    mn = torch.empty(d, dtype=torch.float64, device="cuda") if mean else None
    e.multikrum_device_ptr(X.data_ptr(), dt, n, d, X.stride(0), f, sel.data_ptr(),
                           sc.data_ptr() if sc is not None else None,
                           mn.data_ptr() if mn is not None else None)
    e.synchronize()
    return (sel.cpu().numpy(), sc.cpu().numpy() if sc is not None else None,
            mn.cpu().numpy() if mn is not None else None)


def _timed_kernels(e, X, f):
    e.timing_enable(True)
    _run(e, X, f)
    t = e.timing_read()
    e.timing_enable(False)
    return t


SMALL = [k for k in GU.small_cases() if GU.C.case_params(k)["n"] <= 128
         and not GU.C.case_params(k)["error"]]


@pytest.mark.parametrize("name", SMALL)
def test_small_goldens_one_launch(name, engine, oracle):
    Xh, p = GU.build_input(name, oracle)
    n, d, f = p["n"], p["d"], p["f"]
    X = torch.from_numpy(np.ascontiguousarray(Xh)).cuda()
    t = _timed_kernels(engine, X, f)
    assert "k_small" in t and "k_gram" not in t, t  # the one-launch path ran
    sel, sc, mean = _run(engine, X, f)
    g = GU.load(name)
    mg = engine.selection_margin()
    GU.check_margin(mg, sc, g["sq"], n, f, d)
    assert mg["near_tie"] == p["tie"]
    if not mg["near_tie"]:
        assert np.array_equal(sel, g["sel"])
    GU.check_scores(sc, g, rel=1e-9)
    if not p["tie"]:
        GU.check_mean(mean, g, GU.manifest()[name])


@pytest.mark.parametrize("n,d,f,dtype", [
    (2, 1, 1, torch.float64), (3, 7, 1, torch.float64), (10, 25, 2, torch.float64),
    (16, 8, 5, torch.float64), (17, 1001, 5, torch.float64), (64, 4096, 20, torch.float64),
    (100, 7850, 30, torch.float64), (100, 7850, 50, torch.float64), (127, 333, 40, torch.float64),
    (128, 65536, 38, torch.float64), (100, 7852, 30, torch.float32), (33, 1003, 10, torch.float32),
    (128, 262144, 38, torch.float64)])
def test_small_matches_general_chain(engine, oracle, n, d, f, dtype):
    from biscotti_amd.krum import Engine
    gen = Engine(0)
    gen.set_stream(torch.cuda.current_stream().cuda_stream)
    gen.set_small_path(False)
    try:
        Xh = oracle.synth(n, d, 300 + n + d, max(1, f // 2),
                          dtype=np.float32 if dtype == torch.float32 else np.float64)
        X = torch.from_numpy(Xh).cuda()
        a = _run(engine, X, f)
        b = _run(gen, X, f)
        assert "k_small" not in _timed_kernels(gen, X, f)
        assert np.array_equal(a[0], b[0])
        assert np.array_equal(a[2].view(np.uint8), b[2].view(np.uint8))  # mean: same order
        scale = max(1e-300, float(np.max(np.abs(b[1]))))
        assert float(np.max(np.abs(a[1] - b[1]))) <= 1e-12 * scale
        osel, osc, omean = oracle.krum(Xh, f)
        assert np.array_equal(a[0], osel)
        assert float(np.max(np.abs(a[1] - osc))) <= 1e-9 * max(1e-300, float(np.max(np.abs(osc))))
    finally:
        gen.close()


def test_small_many_launches_alternating_shapes(engine, oracle):
    """Back-to-back launches over alternating shapes, without syncs in between
    (the queue counters reset at the end of every launch, in stream order);
    every result bitwise equal to a lone call's."""
    shapes = [(10, 25, 2), (100, 7850, 30), (128, 1000, 60), (37, 513, 11)]
    data, ref = [], []
    for i, (n, d, f) in enumerate(shapes):
        X = torch.from_numpy(oracle.synth(n, d, 70 + i, f)).cuda()
        data.append(X)
        ref.append(_run(engine, X, f))
    outs = []
    for r in range(60):
        i = r % len(shapes)
        n, d, f = shapes[i]
        X = data[i]
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        sc = torch.empty(n, dtype=torch.float64, device="cuda")
        mn = torch.empty(d, dtype=torch.float64, device="cuda")
        engine.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(),
                                    sc.data_ptr(), mn.data_ptr())
        outs.append((i, sel, sc, mn))
    engine.synchronize()
    for i, sel, sc, mn in outs:
        for u, v in zip((sel.cpu().numpy(), sc.cpu().numpy(), mn.cpu().numpy()), ref[i]):
            assert np.array_equal(u.view(np.uint8), v.view(np.uint8))
    engine.selection_margin()  # raises (BK_EHIP) if any hand-off wait had timed out


def test_small_optional_outputs(engine, oracle):
    Xh = oracle.synth(100, 7850, 5, 30)
    X = torch.from_numpy(Xh).cuda()
    full = _run(engine, X, 30)
    s1, _, _ = _run(engine, X, 30, scores=False, mean=False)
    assert np.array_equal(s1, full[0])
    s2, _, m2 = _run(engine, X, 30, scores=False)
    assert np.array_equal(m2.view(np.uint8), full[2].view(np.uint8))


def test_timing_stride_samples_launches(engine, oracle):
    """bk_timing_stride: the bench's timed region events every 10th k_small."""
    n, d, f = 40, 300, 10
    X = oracle.synth(n, d, 11, 8)
    Xd = torch.from_numpy(X).cuda()
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    try:
        engine.timing_select(["k_small"])
        engine.timing_stride(4)
        for _ in range(9):
            engine.multikrum_device_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr())
        engine.synchronize()
        t = engine.timing_read()
        assert t["k_small"]["count"] == 3  # launches 0, 4, 8
    finally:
        engine.timing_stride(1)
        engine.timing_select([])


@pytest.mark.parametrize("n,d,f,dtype", [(100, 7850, 30, np.float64), (10, 25, 2, np.float64),
                                         (128, 4097, 38, np.float64), (33, 1003, 10, np.float32)])
def test_host_entry_writes_outputs_in_place(engine, oracle, n, d, f, dtype):
    """The synchronous host entry at n <= 128: k_small / k_tiny write sel,
    scores, mean and the margin record straight into a mapped pinned block
    (no device-to-host copy).  Bitwise the device entry's outputs, the same
    margin record, and bk_selection_margin follows whichever call was last."""
    Xh = oracle.synth(n, d, 900 + n, max(1, f // 2), dtype=dtype)
    other = oracle.synth(n, d, 901 + n, max(1, f // 2), dtype=dtype)
    hs, hsc, hm = engine.multikrum(Xh, f)
    hmg = engine.selection_margin()
    ds, dsc, dm = _run(engine, torch.from_numpy(Xh).cuda(), f)
    dmg = engine.selection_margin()
    assert np.array_equal(hs, ds)
    assert np.array_equal(hsc.view(np.uint8), dsc.view(np.uint8))
    assert np.array_equal(hm.view(np.uint8), dm.view(np.uint8))
    assert hmg == dmg
    osel, _, _ = oracle.krum(Xh, f)
    assert np.array_equal(hs, osel)
    # a device call on another batch, then the host entry again: each margin
    # read returns the last call's record, wherever it lives
    _run(engine, torch.from_numpy(other).cuda(), f)
    omg = engine.selection_margin()
    engine.multikrum(Xh, f)
    assert engine.selection_margin() == hmg
    assert omg != hmg


@pytest.mark.parametrize("dtype,n,d,ld,f", [
    (np.float64, 12, 3, 4, 4),         # a numpy view X[:, :3] of an n x 4 array: ld == dld != d
    (np.float64, 100, 7849, 7850, 30),  # mnist-sized, odd d
    (np.float32, 20, 6, 8, 5),
    (np.float32, 64, 1021, 1024, 20),
    (np.float64, 10, 25, 26, 2)])       # config A's shape (k_tiny), padded
def test_host_small_strided_view(engine, oracle, dtype, n, d, ld, f):
    """the host entry of the n <= 128 path with ld equal to
    the 16-B-rounded d but d itself shorter.  The batch must cross as a 2-D
    copy; a linear n*d copy shifted every row after the first."""
    full = oracle.synth(n, ld, 900 + n + d, f, dtype=dtype)
    Xv = full[:, :d]
    assert Xv.strides[0] // Xv.itemsize == ld
    sel, sc, mean = engine.multikrum(Xv, f)
    osel, osc, omean = oracle.krum(np.ascontiguousarray(Xv), f)
    assert np.array_equal(sel, osel)
    assert np.max(np.abs(sc - osc)) <= 1e-9 * max(1e-300, np.max(np.abs(osc)))
    mscale = float(np.max(np.mean(np.abs(Xv[osel].astype(np.float64)), axis=0)))
    assert np.max(np.abs(mean - omean)) <= 1e-9 * max(mscale, 1e-300)


HOST_SHAPES = [
    (100, 7850, 30, np.float64, 0),   # config B (mnist): 62 chunks
    (100, 7849, 30, np.float64, 1),   # odd d, padded host rows
    (128, 2048, 60, np.float32, 0),   # the smallest pipelined batch (16 chunks)
    (37, 30001, 11, np.float64, 0),
    (64, 4099, 20, np.float32, 3)]


def _host_entry_check(engine, oracle, n, d, f, dtype, pad, launches):
    """bk_multikrum from a host batch (pageable, then pinned) against the
    device-resident one-launch call on the same rows: selection, scores and
    mean bitwise; `launches` k_small launches and (one launch) one H2D."""
    import ctypes
    full = oracle.synth(n, d + pad, 4000 + n + d, f, dtype=dtype)
    Xv = full[:, :d]
    ref = _run(engine, torch.from_numpy(np.ascontiguousarray(Xv)).cuda(), f)
    engine.timing_enable(True)
    got = engine.multikrum(Xv, f)  # pageable
    t = engine.timing_read()
    engine.timing_enable(False)
    assert t["k_small"]["count"] == launches, t
    assert ("h2d" in t) == (launches == 1), t
    for u, v in zip(got, ref):
        assert np.array_equal(u.view(np.uint8), v.view(np.uint8))
    # pinned (the verifier's stage_alloc buffers)
    Xp = torch.from_numpy(np.ascontiguousarray(full)).pin_memory()
    m = n - f
    sel = np.empty(m, dtype=np.int64)
    sc = np.empty(n, dtype=np.float64)
    mean = np.empty(d, dtype=np.float64)
    mo = ctypes.c_int64(0)
    dt = _lib.BK_F32 if dtype == np.float32 else _lib.BK_F64
    _lib.check(_lib.lib().bk_multikrum(engine.ctx, ctypes.c_void_p(Xp.data_ptr()),
                                       _lib.BK_HOST_PINNED, dt, n, d, d + pad, f, sel.ctypes.data,
                                       ctypes.addressof(mo), sc.ctypes.data, mean.ctypes.data))
    for u, v in zip((sel, sc, mean), ref):
        assert np.array_equal(u.view(np.uint8), v.view(np.uint8))
    engine.selection_margin()  # the S + M launch's record is readable (no hand-off error)


@pytest.mark.parametrize("n,d,f,dtype,pad", HOST_SHAPES)
def test_host_entry_bitwise(engine, oracle, n, d, f, dtype, pad):
    """The default host entry for n <= 128: one H2D of the batch, one k_small
    launch; bitwise the device call's outputs."""
    _host_entry_check(engine, oracle, n, d, f, dtype, pad, launches=1)


def test_host_entry_pipelined_bitwise():
    """VERDICT r3 item 7, the A/B form (BK_SMALL_PIPE=4, read at bk_create,
    so in a child process): the batch crosses PCIe in 4 column chunks on the
    copy stream, each chunk's G items launch as soon as it lands, then one
    S + M launch: the same items and partials as the one-launch call, so
    every output is bitwise the device call's.  (Slower than one copy at
    config B, 0.234 vs 0.157 ms per call: not the default)"""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    body = r"""
import sys, os, json
sys.path.insert(0, %r); sys.path.insert(0, os.path.join(%r, "tests"))
sys.path.insert(0, os.path.join(%r, "tests", "golden"))
import numpy as np, torch
from biscotti_amd.krum import Engine
from oracle import oracle as O
import test_gpu_small as T
eng = Engine(0)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
for shp in T.HOST_SHAPES:
    T._host_entry_check(eng, O, *shp, launches=5)
print(json.dumps({"ok": True}))
""" % (repo, repo, repo)
    e = dict(os.environ, BK_SMALL_PIPE="4")
    r = subprocess.run([sys.executable, "-c", body], env=e, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["ok"]
