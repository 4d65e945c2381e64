"""Golden-case catalogue shared by gen_goldens.py (run once, in the survey/build
container, against the imported reference) and by the tests (run anywhere).

Each case names its synthetic input (spec: DESIGN.md "Synthetic inputs") plus
optional edge-case modifications, so the GPU box can rebuild the exact input
without the reference.  Configs A-E are BASELINE.json's configs; seeds are
20261015 + config id.
"""
import numpy as np

SEED0 = 20261015
FP32ROUND = 1

# name: dict(n, d, f, seed, nbyz, [mu_scale, byz_scale, sigma, flags, dtype, mods, large])
CASES = {
    # --- BASELINE.json configs -------------------------------------------------
    "A_creditcard": dict(n=10, d=25, f=2, seed=SEED0 + 1, nbyz=2),
    "B_mnist": dict(n=100, d=7850, f=30, seed=SEED0 + 2, nbyz=30, flags=FP32ROUND),
    "C_1024x131072": dict(n=1024, d=131072, f=307, seed=SEED0 + 3, nbyz=307, large=True),
    "D_512x1M_f153": dict(n=512, d=1048576, f=153, seed=SEED0 + 4, nbyz=153, large=True),
    "D_512x1M_f256": dict(n=512, d=1048576, f=256, seed=SEED0 + 4, nbyz=153, large=True),
    "E_4096x262144_fp32": dict(n=4096, d=262144, f=1228, seed=SEED0 + 5, nbyz=1228,
                               dtype="float32", large=True),
    # --- the deployed verifier's real shape: localTest.sh creditcard, n<=4, k=0 -
    "A_n4_k0_tie": dict(n=4, d=25, f=2, seed=SEED0 + 11, nbyz=1, tie=True),
    # --- edge cases the reference's semantics define ---------------------------
    "edge_n2_f1": dict(n=2, d=16, f=1, seed=SEED0 + 12, nbyz=0, tie=True),
    "edge_n3_f1": dict(n=3, d=16, f=1, seed=SEED0 + 13, nbyz=1, tie=True),
    "edge_k1": dict(n=5, d=64, f=2, seed=SEED0 + 14, nbyz=1),
    "edge_zeros_tie": dict(n=8, d=32, f=3, seed=SEED0 + 15, nbyz=0, mods=[("zeros",)], tie=True),
    "edge_f0_error": dict(n=10, d=25, f=0, seed=SEED0 + 16, nbyz=0, error=True),
    "honest_boundary": dict(n=64, d=4096, f=20, seed=SEED0 + 17, nbyz=5),
    "dup_rows": dict(n=32, d=1000, f=8, seed=SEED0 + 18, nbyz=8, mods=[("dup", 3, 17), ("dup", 9, 30)]),
    "nan_row": dict(n=24, d=500, f=6, seed=SEED0 + 19, nbyz=6, mods=[("nan", 5, 7)]),
    "inf_row": dict(n=24, d=500, f=6, seed=SEED0 + 20, nbyz=6, mods=[("inf", 11, 3)]),
    "outliers_1e6": dict(n=40, d=2000, f=12, seed=SEED0 + 21, nbyz=12, byz_scale=1e6),
    "half_clip": dict(n=50, d=2048, f=25, seed=SEED0 + 22, nbyz=20),
    "ragged_67x1003": dict(n=67, d=1003, f=20, seed=SEED0 + 23, nbyz=20),
    "fp32_200x3000": dict(n=200, d=3000, f=60, seed=SEED0 + 24, nbyz=60, dtype="float32"),
    "n1000_d2000": dict(n=1000, d=2000, f=300, seed=SEED0 + 25, nbyz=250),
    "n2500_d512": dict(n=2500, d=512, f=700, seed=SEED0 + 26, nbyz=600),
    "n129_d4097": dict(n=129, d=4097, f=40, seed=SEED0 + 27, nbyz=40),
    # --- the selection boundary INSIDE the honest cluster (nbyz < f): honest
    #     rows are rejected too, and the boundary gap is a tiny fraction of the
    #     scores (the A-E goldens separate a 50-sigma Byzantine
    #     cluster, which any Gram within ~1e-3 would select identically) ---------
    "B_tight": dict(n=100, d=7850, f=30, seed=SEED0 + 31, nbyz=10, flags=FP32ROUND),
    "C_tight": dict(n=1024, d=131072, f=307, seed=SEED0 + 32, nbyz=200, large=True),
    "E_tight_fp32": dict(n=4096, d=262144, f=1228, seed=SEED0 + 33, nbyz=800, dtype="float32",
                         large=True),
    "fp32_tight_700x65536": dict(n=700, d=65536, f=210, seed=SEED0 + 34, nbyz=100,
                                 dtype="float32", large=True),
}

MEAN_FULL_MAX_D = 8192   # store the full mean up to this d; sampled coords above
MEAN_SAMPLES = 4096
MEAN_BLOCKS = 64


def case_params(name):
    c = dict(CASES[name])
    c.setdefault("mu_scale", 0.01)
    c.setdefault("byz_scale", 0.05)
    c.setdefault("sigma", 1e-3)
    c.setdefault("flags", 0)
    c.setdefault("dtype", "float64")
    c.setdefault("mods", [])
    c.setdefault("large", False)
    c.setdefault("tie", False)
    c.setdefault("error", False)
    return c


def apply_mods(X, mods):
    for mod in mods:
        kind = mod[0]
        if kind == "zeros":
            X[...] = 0
        elif kind == "dup":
            X[mod[2]] = X[mod[1]]
        elif kind == "nan":
            X[mod[1], mod[2]] = np.nan
        elif kind == "inf":
            X[mod[1], mod[2]] = np.inf
        else:
            raise ValueError(kind)
    return X


def sample_cols(d, seed):
    """Deterministic sample of mean coordinates checked for large d."""
    rng = np.random.default_rng(seed)
    k = min(MEAN_SAMPLES, d)
    return np.sort(rng.choice(d, size=k, replace=False)).astype(np.int64)


def mean_blocks(mean):
    """Sums of MEAN_BLOCKS contiguous column blocks (ascending, sequential)."""
    d = len(mean)
    edges = np.linspace(0, d, MEAN_BLOCKS + 1).astype(np.int64)
    return np.array([np.sum(mean[edges[i]:edges[i + 1]]) for i in range(MEAN_BLOCKS)]), edges
