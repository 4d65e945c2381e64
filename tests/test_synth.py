"""The synthetic-batch spec is implemented three times (numpy, C oracle, HIP);
the CPU side checks numpy == C bit-for-bit here, the GPU side is checked in
tests/test_gpu_parity.py."""
import numpy as np
import pytest

import synth_np as S


@pytest.mark.parametrize("n,d,nbyz,flags,dt", [
    (10, 25, 2, 0, np.float64), (100, 785, 30, 1, np.float64), (37, 300, 5, 0, np.float32),
    (1, 7, 0, 0, np.float64), (64, 129, 64, 1, np.float32)])
def test_numpy_equals_c(oracle, n, d, nbyz, flags, dt):
    a = oracle.synth(n, d, 1234 + n, nbyz, flags=flags, dtype=dt)
    b = S.synth(n, d, 1234 + n, nbyz, flags=flags, dtype=dt)
    assert a.dtype == b.dtype
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_column_shards_compose(oracle):
    full = oracle.synth(16, 1000, 99, 4)
    parts = [oracle.synth(16, 1000, 99, 4, c0=c0, dl=dl, d_total=1000)
             for c0, dl in [(0, 256), (256, 512), (768, 232)]]
    assert np.array_equal(np.concatenate(parts, axis=1), full)


def test_perm_is_a_permutation(oracle):
    for n in (1, 2, 10, 513):
        p = oracle.synth_perm(5, n)
        assert sorted(p.tolist()) == list(range(n))
        assert np.array_equal(p, S.synth_perm(5, n))


def test_byzantine_rows_are_shifted(oracle):
    n, d, nbyz = 40, 4000, 10
    X = oracle.synth(n, d, 3, nbyz)
    perm = oracle.synth_perm(3, n)
    byz = perm >= n - nbyz
    mu = X[~byz].mean(0)
    dist = np.linalg.norm(X - mu, axis=1)
    assert dist[byz].min() > 3 * dist[~byz].max()
