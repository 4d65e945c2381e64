"""CPU: the §8(f) rows-2/3 oracle (oracle/aggregate_oracle.c) against known
answers and an independent pure-Python restatement of the Go loops, plus the
host-side stake bookkeeping of create_block.  No GPU.

Reference: DistSys/honest.go:346-381 (createBlock), DistSys/kyber.go:698-757
(updateFloatToInt / updateIntToFloat), DistSys/main.go:1524-1537, 1606-1653
(noise).  Parity of these restatements is unpinned by the reference itself (no
Go toolchain here, no reference tests for them): see DESIGN.md §2.
"""
import numpy as np
import pytest

from oracle import oracle as O

I64_MIN = -(1 << 63)


def py_go_i64(y):
    # Go amd64 int64(float64): truncate toward zero; NaN / out of range -> MinInt64
    if y != y or not (-9223372036854775808.0 <= y < 9223372036854775808.0):
        return I64_MIN
    return int(y)  # Python int() truncates toward zero


def wrap64(v):
    return ((v + (1 << 63)) % (1 << 64)) - (1 << 63)


@pytest.mark.parametrize("y,want", [
    (0.0, 0), (-0.0, 0), (1.9999, 1), (-1.9999, -1), (-0.5, 0), (1234.4999999999998, 1234),
    (float("nan"), I64_MIN), (float("inf"), I64_MIN), (float("-inf"), I64_MIN),
    (9223372036854775808.0, I64_MIN), (-9223372036854775808.0, I64_MIN),
    (9223372036854774784.0, 9223372036854774784), (-9223372036854774784.0, -9223372036854774784),
    (1e300, I64_MIN),
])
def test_go_f64_to_i64_known_answers(y, want):
    assert O.go_f64_to_i64(y) == want
    assert py_go_i64(y) == want


def test_qsum_known_answer():
    # updateFloatToInt with PRECISION = 4 (main.go:45): 0.12345 * 1e4 = 1234.4999999999998
    X = np.array([[0.12345, -0.00019, 2.5], [0.00005, 0.00019, -2.5]])
    s, sf = O.qsum(X, [0, 1], 4)
    assert s.tolist() == [1234 + 0, -1 + 1, 25000 - 25000]
    assert sf.tolist() == [0.1234, 0.0, 0.0]


def _rand(n, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d)) * 10.0 ** rng.integers(-6, 3, size=(n, 1))
    return X


@pytest.mark.parametrize("precision", [0, 4, 9, 18])
def test_qsum_vs_python(precision):
    X = _rand(7, 33, precision)
    X[2, 3] = np.nan
    X[4, 5] = np.inf
    X[1, 6] = -0.0
    X[5, 7] = 9.2e18 / 10.0 ** precision  # near the int64 edge: sums wrap
    X[6, 7] = 9.2e18 / 10.0 ** precision
    idx = [6, 0, 5, 5, 2, 4]
    s, sf = O.qsum(X, idx, precision)
    scale = 10.0 ** precision
    assert scale == float(10 ** precision)  # exact for p <= 22
    for c in range(X.shape[1]):
        acc = 0
        for r in idx:
            acc = wrap64(acc + py_go_i64(X[r, c] * scale))
        assert s[c] == acc, c
        assert sf[c] == float(acc) / scale, c


def test_aggregate_vs_python():
    X = _rand(9, 41, 1)
    g0 = _rand(1, 41, 2)[0]
    idx = [3, 0, 8, 3, 5]
    got = O.aggregate(X, idx, g0)
    for c in range(41):
        v = float(g0[c])
        for r in idx:
            v = v + float(X[r, c])
        assert got[c] == v or (v != v and got[c] != got[c])
    assert np.array_equal(O.aggregate(X, [], g0), g0)


def test_aggregate_order_matters():
    # sequential fp64 adds are not associative: the oracle keeps the Go order
    X = np.array([[1e16], [1.0], [-1e16]])
    assert O.aggregate(X, [0, 1, 2], np.zeros(1))[0] == 0.0
    assert O.aggregate(X, [0, 2, 1], np.zeros(1))[0] == 1.0


@pytest.mark.parametrize("k", [0, 1, 3, 9])
def test_noise_vs_python(k):
    rng = np.random.default_rng(k)
    D = rng.standard_normal((3, 17))
    N = rng.standard_normal((3, k, 17)) * 1e-3
    if k:
        N[1, 0, 2] = -0.0
    got = O.noise(D, N)
    for i in range(3):
        for c in range(17):
            s = 0.0
            for j in range(k):
                s += float(N[i, j, c])
            s = s / float(k) if k else float("nan")
            want = float(D[i, c]) + s
            assert got[i, c] == want or (want != want and got[i, c] != got[i, c])


def test_create_block_stakes_without_accepted():
    # host bookkeeping only (no accepted update -> no GPU call), honest.go:364-369
    from biscotti_amd.aggregate import STAKE_UNIT, create_block
    from biscotti_amd.krum import Update
    ups = [Update(SourceID=3, Delta=np.ones(4)), Update(SourceID=7, Delta=np.ones(4))]
    stake = {3: 10}
    g = create_block(np.arange(4.0), ups, stake)
    assert np.array_equal(g, np.arange(4.0))
    assert stake == {3: 10 - STAKE_UNIT, 7: -STAKE_UNIT}
