"""Host-side logic that needs no GPU: sharding, the packed-upper layout, the
reference-mirroring verifier bookkeeping."""
import numpy as np
import pytest

from biscotti_amd import dist as D
from biscotti_amd.krum import KRUMValidator, Update


@pytest.mark.parametrize("d,world", [(1 << 20, 1), (1 << 20, 8), (7850, 3), (25, 4), (1003, 8),
                                     (8, 8)])
def test_shards_partition_columns(d, world):
    sh = D.all_shards(d, world)
    pos = 0
    for c0, dl in sh:
        assert c0 == pos or dl == 0
        assert dl >= 0
        if dl:
            assert c0 % D.ALIGN == 0
        pos = c0 + dl if dl else pos
    assert sum(dl for _, dl in sh) == d


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    for n in (1, 5, 64, 65, 130):
        A = rng.standard_normal((n, 7))
        G = A @ A.T
        U = D.pack_upper(G, 7)
        assert U.size == D.upper_elems(n)
        assert U[-4] == 7.0 and U[-3] == 0.0 and U[-2] == 0.0 and U[-1] == 0.0
        assert np.allclose(D.unpack_upper(U, n), G)


def test_packed_partials_sum_to_full_gram(oracle):
    X = oracle.synth(70, 1000, 11, 10)
    full = D.pack_upper(oracle.gram(X), 1000)
    parts = sum(D.pack_upper(oracle.gram(np.ascontiguousarray(X[:, c0:c0 + dl])), dl)
                for c0, dl in D.all_shards(1000, 3))
    assert np.allclose(parts, full, rtol=1e-12, atol=1e-15)
    assert parts[-4] == 1000.0  # the trailing record sums to the total column count
    assert parts[-3] == 0.0     # ... none of it on the fp32 MFMA
    assert parts[-2] == 0.0     # ... nor int8-sliced


def test_pack_upper_needs_a_column_count():
    with pytest.raises(ValueError):
        D.pack_upper(np.eye(3), None)


def test_validator_bookkeeping_mirrors_krum_go():
    v = KRUMValidator()
    assert v.NumAdversaries == 0.5
    v.UpdateList = [Update(SourceID=s) for s in (4, 7, 9, 12)]
    v.AcceptedList = [1, 3]
    assert v.check_if_accepted(7) and v.check_if_accepted(12)
    assert not v.check_if_accepted(4) and not v.check_if_accepted(99)
    v.flush_collected_updates(collecting_updates=True)
    assert v.UpdateList
    v.flush_collected_updates()
    assert v.UpdateList == [] and v.AcceptedList == []


def test_clip_rule_matches_krum_go():
    # krum.go:110: adversaryCount := int(krumval.NumAdversaries * float64(numUpdates))
    for n, clip in [(4, 2), (5, 2), (10, 5), (7, 3), (1, 0), (100, 50)]:
        assert int(0.5 * float(n)) == clip


def test_krum_rejects_clip_zero_like_numpy():
    from biscotti_amd.krum import krum
    with pytest.raises(ValueError):
        krum(np.zeros((3, 4)), 0)
    with pytest.raises(ValueError):
        krum(np.zeros((3, 4)), 3)
