"""The oracle (oracle/krum_oracle.c) pinned against the reference's own outputs.

Goldens were produced by running the reference numpy krum/get_krum_scores
(ML/code/logistic_validator.py:36-65) on the same inputs; see
tests/golden/gen_goldens.py.  Selection must match bit-exactly, scores to
rounding (the reference's Gram is BLAS-rounded), the mean within 1e-9 of the
norm-wise scale, and the row norms np.sum(X**2, 1) bit-exactly (the oracle
restates numpy's pairwise summation).
"""
import numpy as np
import pytest

import golden_util as GU


@pytest.mark.parametrize("name", GU.small_cases())
def test_oracle_matches_reference_golden(name, oracle):
    X, p = GU.build_input(name, oracle)
    rec = GU.manifest()[name]
    if p["error"]:
        assert rec["error"] == "ValueError"
        with pytest.raises(ValueError):
            oracle.krum(X, p["f"])
        return
    g = GU.load(name)
    sel, sc, mean = oracle.krum(X, p["f"])
    assert np.array_equal(sel, g["sel"]), (sel, g["sel"])
    if p["tie"]:
        # numpy's introselect is implementation-defined on ties; the reference
        # happened to pick the lowest indices here, which is also our rule
        assert np.array_equal(sel, np.arange(len(sel)))
    GU.check_scores(sc, g, rel=1e-12)
    GU.check_mean(mean, g, rec)
    sq = oracle.sqnorms(X)
    assert np.array_equal(sq, g["sq"], equal_nan=True), "np.sum(X**2, 1) restatement not bit-exact"


@pytest.mark.parametrize("name", [n for n in GU.small_cases() if GU.C.CASES[n]["n"] <= 128 and not GU.C.case_params(n)["error"]])
def test_oracle_distance_matrix(name, oracle):
    X, p = GU.build_input(name, oracle)
    g = GU.load(name)
    n = p["n"]
    _, D = oracle.krum_scores(X, n - p["f"], want_D=True)
    ref = g["D"]
    assert np.array_equal(np.isnan(D), np.isnan(ref))
    fin = np.isfinite(ref)
    scale = max(1e-300, np.max(np.abs(ref[fin]))) if fin.any() else 1
    # |D_ij| carries the cancellation of ||x_i||^2 + ||x_j||^2 - 2<x_i,x_j>; bound by the norms
    sq = g["sq"]
    bound = 1e-13 * (np.abs(sq)[:, None] + np.abs(sq)[None, :])
    assert np.all(np.abs(D[fin] - ref[fin]) <= bound[fin] + 1e-300), scale


def test_margins_recorded():
    man = GU.manifest()
    for name in GU.small_cases():
        rec = man[name]
        if rec.get("error"):
            continue
        assert rec["m"] == GU.C.CASES[name]["n"] - GU.C.CASES[name]["f"]
        assert rec["gap"] >= 0 or np.isnan(rec["gap"])


@pytest.mark.slow
@pytest.mark.parametrize("name", [n for n in GU.large_cases() if n.startswith("C_")])
def test_oracle_large_config_C(name, oracle):
    X, p = GU.build_input(name, oracle)
    g = GU.load(name)
    sel, sc, mean = oracle.krum(X, p["f"])
    assert np.array_equal(sel, g["sel"])
    GU.check_scores(sc, g, rel=1e-11)
    GU.check_mean(mean, g, GU.manifest()[name])
