"""CPU: the RONI oracle (oracle/roni_oracle.c) against the goldens produced by
the reference roni (ML/code/logistic_validator.py:22-33; gen_roni_goldens.py):
scores bit-exact.  No GPU."""
import numpy as np
import pytest

import roni_util as RU


@pytest.mark.parametrize("name", RU.names())
def test_roni_oracle_matches_reference_goldens(oracle, name):
    Xv, yv, ww, deltas, want = RU.load(name)
    got = oracle.roni(Xv, yv, ww, deltas)
    assert np.array_equal(got.view(np.int64), want.view(np.int64)), (name, got, want)


def test_roni_oracle_semantics():
    from oracle import oracle as O
    Xv = np.array([[1.0, 0.0], [0.0, 0.0], [1.0, 1.0]])
    yv = np.array([1.0, 0.0, -1.0])
    # row 1 dots to 0: sign 0 == label 0 (no error); NaN weights -> every row errs
    s = O.roni(Xv, yv, np.array([1.0, 0.0]), np.array([[0.0, 0.0], [np.nan, 0.0], [-2.0, 0.0]]))
    assert s[0] == 0.0
    assert s[1] == 3 / 3 - 1 / 3
    assert s[2] == 1 / 3 - 1 / 3  # w = [-1, 0]: row 0 now wrong, row 2 now right
