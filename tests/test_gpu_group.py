"""One process, G GPUs (bk_group_*) on an MI355X.

The GPU box has one device, so the G > 1 cases run G contexts on device 0
with the host exchange (BK_GROUP_HOST_EXCHANGE: partial Grams summed in fixed
rank order through pinned host memory, bitwise the order of the RCCL
deterministic mode).  That exercises the sharding, the per-device H2D of
column shards, the exchange and the scattered mean exactly as on G devices;
the RCCL group modes run at G = 1 (ncclCommInitAll on one device).
"""
import numpy as np
import pytest

import golden_util as GU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402
from biscotti_amd.dist import shard_bounds  # noqa: E402
from biscotti_amd.krum import GroupEngine  # noqa: E402


@pytest.mark.parametrize("mode", [_lib.BK_GROUP_ALLREDUCE, _lib.BK_GROUP_DETERMINISTIC,
                                  _lib.BK_GROUP_HOST_EXCHANGE])
def test_group_of_one_equals_engine_bitwise(engine, oracle, mode):
    X = oracle.synth(300, 5000, 11, 90)
    g = GroupEngine([0], mode)
    try:
        a = g.multikrum(X, 90)
    finally:
        g.close()
    b = engine.multikrum(X, 90)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("n,d,f", [(100, 7850, 30), (300, 1003, 90), (64, 8 * 8 + 5, 20),
                                   (1100, 2003, 50)])
def test_group_host_exchange_matches_oracle(engine, oracle, G, n, d, f):
    """G contexts on device 0: the selection equals the single-context one and
    the oracle's; the mean is column-local, so it is bitwise the single-context
    mean (same selection, same per-column order of adds)."""
    X = oracle.synth(n, d, 100 + G, f)
    g = GroupEngine([0] * G, _lib.BK_GROUP_HOST_EXCHANGE)
    try:
        assert g.size == G
        sel, sc, mean = g.multikrum(X, f)
    finally:
        g.close()
    osel, osc, omean = oracle.krum(X, f)
    esel, esc, emean = engine.multikrum(X, f)
    assert np.array_equal(sel, osel) and np.array_equal(sel, esel)
    assert float(np.max(np.abs(sc - osc))) <= 1e-11 * float(np.max(np.abs(osc)))
    assert np.array_equal(mean, emean)
    scale = float(np.max(np.mean(np.abs(X[osel]), axis=0)))
    assert float(np.max(np.abs(mean - omean))) <= 1e-9 * scale
    # (64 x 69 at G = 8 leaves ranks 5-7 without columns: that call takes the
    # one-device path, and must agree all the same; 1100 x 2003 with m = 1050
    # takes K4's row segments, whose order depends on m only, so each device's
    # few columns add exactly as the single context's)


def test_group_small_d_falls_back_to_one_device(engine, oracle):
    X = oracle.synth(40, 12, 3, 10)  # d = 12 < 8 * G: a shard would be empty
    assert shard_bounds(12, 4, 3)[1] == 0
    g = GroupEngine([0] * 4, _lib.BK_GROUP_HOST_EXCHANGE)
    try:
        a = g.multikrum(X, 10)
    finally:
        g.close()
    b = engine.multikrum(X, 10)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_group_goldens_fp32(oracle):
    """Two golden cases through a 2-context group, one in fp32."""
    for name in ("B_mnist", "fp32_200x3000"):
        X, p = GU.build_input(name, oracle)
        g = GroupEngine([0, 0], _lib.BK_GROUP_HOST_EXCHANGE)
        try:
            sel, sc, mean = g.multikrum(X, p["f"])
        finally:
            g.close()
        gl = GU.load(name)
        assert np.array_equal(sel, gl["sel"]), name
        GU.check_scores(sc, gl, rel=1e-9)
        GU.check_mean(mean, gl, GU.manifest()[name])


def test_group_errors():
    with pytest.raises(ValueError):
        GroupEngine([0, 0], _lib.BK_GROUP_ALLREDUCE)  # RCCL needs distinct devices
    g = GroupEngine([0], _lib.BK_GROUP_HOST_EXCHANGE)
    try:
        with pytest.raises(ValueError):
            g.multikrum(np.zeros((10, 10)), 0)  # f = 0: the reference's ValueError
    finally:
        g.close()
