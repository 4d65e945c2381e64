"""bk_graph_enable: bk_multikrum_device replayed as a hipGraph.

* eager, capture and replay calls give bitwise the eager results, and a replay
  reads the live batch (new data in the same buffer -> new result);
* a workspace reallocation by a larger call retires the graph (no replay over
  freed buffers): the first signature stays correct afterwards;
* per-kernel timing bypasses the graph (every kernel still evented).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402


def _bufs(n, d, f):
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    return (X, torch.empty(n - f, dtype=torch.int64, device="cuda"),
            torch.empty(n, dtype=torch.float64, device="cuda"),
            torch.empty(d, dtype=torch.float64, device="cuda"))


def _call(e, X, sel, sc, mean, f):
    n, d = X.shape
    e.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, X.stride(0), f, sel.data_ptr(),
                           sc.data_ptr(), mean.data_ptr())
    e.synchronize()
    return sel.cpu().numpy().copy(), sc.cpu().numpy().copy(), mean.cpu().numpy().copy()


@pytest.fixture()
def graph_engine():
    from biscotti_amd.krum import Engine
    e = Engine(0)
    e.set_stream(torch.cuda.current_stream().cuda_stream)
    e.graph_enable(True)
    yield e
    e.close()


def _same(a, b):
    return all(np.array_equal(u.view(np.uint8), v.view(np.uint8)) for u, v in zip(a, b))


@pytest.mark.parametrize("n,d,f", [(100, 7850, 30), (512, 65536, 153), (65, 1001, 20)])
def test_replay_is_bitwise_eager_and_reads_live_data(engine, graph_engine, oracle, n, d, f):
    X, sel, sc, mean = _bufs(n, d, f)
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 11, f)
    ref = _call(engine, X, sel, sc, mean, f)
    for _ in range(4):  # eager, capture, replay, replay
        assert _same(_call(graph_engine, X, sel, sc, mean, f), ref)
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 12, f)  # new batch, same buffer
    got = _call(graph_engine, X, sel, sc, mean, f)
    ref2 = _call(engine, X, sel, sc, mean, f)
    assert _same(got, ref2)
    osel, _, _ = oracle.krum(X.cpu().numpy(), f)
    assert np.array_equal(got[0], osel)


def test_workspace_growth_retires_graphs(engine, graph_engine):
    small = _bufs(64, 4096, 20)
    engine.synth_fill_ptr(small[0].data_ptr(), _lib.BK_F64, 64, 4096, 4096, 0, 4096, 3, 20)
    ref = _call(engine, *small, 20)
    for _ in range(3):
        assert _same(_call(graph_engine, *small, 20), ref)
    big = _bufs(700, 20000, 210)  # grows the context's workspace (plan slabs, U, ...)
    engine.synth_fill_ptr(big[0].data_ptr(), _lib.BK_F64, 700, 20000, 20000, 0, 20000, 4, 210)
    refb = _call(engine, *big, 210)
    for _ in range(3):
        assert _same(_call(graph_engine, *big, 210), refb)
    for _ in range(3):  # the small signature again: recaptured over the new workspace
        assert _same(_call(graph_engine, *small, 20), ref)


def test_timing_bypasses_graph(engine, graph_engine):
    n, d, f = 100, 7850, 30
    X, sel, sc, mean = _bufs(n, d, f)
    engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 5, f)
    ref = _call(engine, X, sel, sc, mean, f)
    for _ in range(3):
        _call(graph_engine, X, sel, sc, mean, f)
    graph_engine.timing_enable(True)
    got = _call(graph_engine, X, sel, sc, mean, f)
    t = graph_engine.timing_read()
    graph_engine.timing_enable(False)
    assert _same(got, ref)
    assert t["k_small"]["count"] == 1  # n <= 128: the one-launch path, evented


def test_replay_after_host_small_call_reports_its_own_margin(graph_engine, oracle):
    """a replayed device call must point the margin readers
    at the record its captured finish writes, and arm bk_synchronize's check --
    not leave them on an earlier host call's output block."""
    n, d, f = 100, 7850, 30
    X, sel, sc, mean = _bufs(n, d, f)
    graph_engine.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 21, f)
    for _ in range(3):  # eager, capture, replay
        _call(graph_engine, X, sel, sc, mean, f)
    rec_dev = graph_engine.selection_margin()
    # a host call of another batch: its record lands in the host output block
    Xh = oracle.synth(90, 333, 5, 20)
    hs, _, _ = graph_engine.multikrum(Xh, 20)
    assert np.array_equal(hs, oracle.krum(Xh, 20)[0])
    rec_host = graph_engine.selection_margin()
    assert rec_host["d"] == 333 and rec_host["k"] == 90 - 20 - 2
    # the replayed device call again: its own record, not the host call's
    got = _call(graph_engine, X, sel, sc, mean, f)
    rec = graph_engine.selection_margin()
    assert rec["d"] == d and rec["k"] == n - f - 2
    assert rec == rec_dev
    assert np.array_equal(got[0], oracle.krum(X.cpu().numpy(), f)[0])
