"""ctypes wrapper for the CPU oracle (oracle/libkrum_oracle.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by biscotti_amd/.  See krum_oracle.c for the
reference file:line each function restates.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libkrum_oracle.so")
_lib = None

_i64 = ctypes.c_int64
_vp = ctypes.c_void_p


def build():
    """Compile the oracle with its Makefile (gcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_check_args.argtypes = [_i64, _i64, _i64]
        L.oracle_check_args.restype = ctypes.c_int
        L.oracle_krum.argtypes = [_vp, ctypes.c_int, _i64, _i64, _i64, _i64, _vp, _vp, _vp]
        L.oracle_krum.restype = _i64
        L.oracle_krum_scores.argtypes = [_vp, ctypes.c_int, _i64, _i64, _i64, _i64, _vp, _vp]
        L.oracle_krum_scores.restype = ctypes.c_int
        L.oracle_gram.argtypes = [_vp, ctypes.c_int, _i64, _i64, _i64, _vp]
        L.oracle_gram.restype = ctypes.c_int
        L.oracle_sqnorms.argtypes = [_vp, ctypes.c_int, _i64, _i64, _i64, _vp]
        L.oracle_sqnorms.restype = ctypes.c_int
        L.oracle_select.argtypes = [_vp, _i64, _i64, _vp]
        L.oracle_select.restype = _i64
        L.oracle_mean.argtypes = [_vp, ctypes.c_int, _i64, _i64, _vp, _i64, _vp]
        L.oracle_mean.restype = None
        L.oracle_synth_fill.argtypes = [_vp, ctypes.c_int, _i64, _i64, _i64, _i64, _i64,
                                        ctypes.c_uint64, _i64, ctypes.c_double, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_int]
        L.oracle_synth_fill.restype = None
        L.oracle_synth_perm.argtypes = [ctypes.c_uint64, _i64, _vp]
        L.oracle_synth_perm.restype = None
        L.oracle_aggregate.argtypes = [_vp, _i64, _i64, _vp, _i64, _vp]
        L.oracle_aggregate.restype = None
        L.oracle_qsum.argtypes = [_vp, _i64, _i64, _vp, _i64, ctypes.c_int, _vp, _vp]
        L.oracle_qsum.restype = None
        L.oracle_noise.argtypes = [_vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _i64]
        L.oracle_noise.restype = None
        L.oracle_roni.argtypes = [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i64, _vp]
        L.oracle_roni.restype = ctypes.c_int
        L.oracle_roni_softmax.argtypes = [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i64,
                                           _i64, _vp, _vp]
        L.oracle_roni_softmax.restype = ctypes.c_int
        L.oracle_roni_softmax_batches.argtypes = [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp,
                                                   _i64, _i64, _vp, _i64, _vp, _vp]
        L.oracle_roni_softmax_batches.restype = ctypes.c_int
        L.oracle_go_f64_to_i64.argtypes = [ctypes.c_double]
        L.oracle_go_f64_to_i64.restype = _i64
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_set_threads.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _x(X):
    X = np.asarray(X)
    if X.dtype not in (np.float64, np.float32):
        X = X.astype(np.float64)
    if X.ndim != 2 or X.strides[1] != X.itemsize:
        X = np.ascontiguousarray(X)
    ld = X.strides[0] // X.itemsize
    return X, int(X.dtype == np.float32), ld


def krum(X, f, want_scores=True, want_mean=True):
    """Returns (sel ascending int64[m], scores float64[n] | None, mean float64[d] | None)."""
    X, is32, ld = _x(X)
    n, d = X.shape
    if lib().oracle_check_args(n, d, f) != 0:
        raise ValueError("invalid Multi-Krum arguments n=%d d=%d f=%d" % (n, d, f))
    m = n - f
    sel = np.empty(m, dtype=np.int64)
    sc = np.empty(n, dtype=np.float64) if want_scores else None
    mean = np.empty(d, dtype=np.float64) if want_mean else None
    r = lib().oracle_krum(_ptr(X), is32, n, d, ld, f, _ptr(sel), _ptr(sc), _ptr(mean))
    if r < 0:
        raise RuntimeError("oracle_krum failed: %d" % r)
    return sel, sc, mean


def krum_scores(X, groupsize, want_D=False):
    X, is32, ld = _x(X)
    n, d = X.shape
    sc = np.empty(n, dtype=np.float64)
    D = np.empty((n, n), dtype=np.float64) if want_D else None
    r = lib().oracle_krum_scores(_ptr(X), is32, n, d, ld, groupsize, _ptr(sc), _ptr(D))
    if r:
        raise RuntimeError("oracle_krum_scores failed: %d" % r)
    return (sc, D) if want_D else sc


def gram(X):
    X, is32, ld = _x(X)
    n, d = X.shape
    G = np.empty((n, n), dtype=np.float64)
    lib().oracle_gram(_ptr(X), is32, n, d, ld, _ptr(G))
    return G


def sqnorms(X):
    X, is32, ld = _x(X)
    n, d = X.shape
    sq = np.empty(n, dtype=np.float64)
    lib().oracle_sqnorms(_ptr(X), is32, n, d, ld, _ptr(sq))
    return sq


def select(scores, m):
    scores = np.ascontiguousarray(scores, dtype=np.float64)
    sel = np.empty(m, dtype=np.int64)
    lib().oracle_select(_ptr(scores), len(scores), m, _ptr(sel))
    return sel


def mean(X, sel):
    X, is32, ld = _x(X)
    n, d = X.shape
    sel = np.ascontiguousarray(sel, dtype=np.int64)
    out = np.empty(d, dtype=np.float64)
    lib().oracle_mean(_ptr(X), is32, d, ld, _ptr(sel), len(sel), _ptr(out))
    return out


def synth(n, d, seed, nbyz, mu_scale=0.01, byz_scale=0.05, sigma=1e-3, flags=0,
          dtype=np.float64, c0=0, dl=None, d_total=None):
    if dl is None:
        dl = d - c0
    if d_total is None:
        d_total = d
    X = np.empty((n, dl), dtype=dtype)
    lib().oracle_synth_fill(_ptr(X), int(X.dtype == np.float32), n, dl, dl, c0, d_total,
                            seed, nbyz, mu_scale, byz_scale, sigma, flags)
    return X


def synth_perm(seed, n):
    p = np.empty(n, dtype=np.int64)
    lib().oracle_synth_perm(seed, n, _ptr(p))
    return p


def set_threads(t):
    lib().oracle_set_threads(int(t))


def num_threads():
    return lib().oracle_num_threads()


# ---- SURVEY.md §8(f) rows 2-3 (oracle/aggregate_oracle.c) -----------------
def _f64(X):
    X = np.asarray(X, dtype=np.float64)
    if X.ndim != 2 or X.strides[1] != 8:
        X = np.ascontiguousarray(X)
    return X, X.strides[0] // 8


def aggregate(X, idx, global_w):
    """honest.go:360-375: returns global_w + X[idx[0]] + X[idx[1]] + ... (sequential)."""
    X, ld = _f64(X)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    out = np.array(global_w, dtype=np.float64, copy=True)
    lib().oracle_aggregate(_ptr(X), X.shape[1], ld, _ptr(idx), len(idx), _ptr(out))
    return out


def qsum(X, idx, precision=4):
    """kyber.go:698-710 + 745-757: (int64 sum, float64 sum) of the quantised rows."""
    X, ld = _f64(X)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    d = X.shape[1]
    s = np.empty(d, dtype=np.int64)
    sf = np.empty(d, dtype=np.float64)
    lib().oracle_qsum(_ptr(X), d, ld, _ptr(idx), len(idx), int(precision), _ptr(s), _ptr(sf))
    return s, sf


def noise(delta, noise_vecs):
    """main.go:1524-1537 + 1606-1653, batched: delta (n, d), noise (n, k, d)."""
    D, ld = _f64(delta)
    N = np.ascontiguousarray(noise_vecs, dtype=np.float64)
    n, d = D.shape
    k = N.shape[1]
    out = np.empty((n, d), dtype=np.float64)
    lib().oracle_noise(_ptr(D), n, d, ld, _ptr(N) if k else None, k, d, _ptr(out), d)
    return out


def go_f64_to_i64(y):
    return lib().oracle_go_f64_to_i64(float(y))


# ---- SURVEY.md §8(f) row 4 (oracle/roni_oracle.c) -------------------------
def roni(Xv, yv, ww, deltas):
    """logistic_validator.py:22-33 for each row of deltas: scores (n,)."""
    Xv = np.ascontiguousarray(Xv, dtype=np.float64)
    yv = np.ascontiguousarray(yv, dtype=np.float64)
    ww = np.ascontiguousarray(ww, dtype=np.float64)
    D = np.ascontiguousarray(np.atleast_2d(deltas), dtype=np.float64)
    nv, d = Xv.shape
    out = np.empty(D.shape[0], dtype=np.float64)
    assert lib().oracle_roni(_ptr(Xv), nv, d, d, _ptr(yv), _ptr(ww), _ptr(D), D.shape[0], d,
                             _ptr(out)) == 0
    return out


def roni_softmax(Xv, yv, n_classes, ww, deltas, near_ties=False):
    """ML/Pytorch/client_obj.py:100-112 (softmax model, getTrainErr) for each
    row of deltas, every update scored on the same sample set (the reference
    with batch_size >= nv): scores (n,).  Xv (nv, d_in) float32, yv (nv,) int
    labels, ww and deltas fp64 of length n_classes * (d_in + 1) ([W row-major,
    b]).  near_ties=True also returns the (n + 1,) near-tie counts (ww, then
    each update's model)."""
    Xv = np.ascontiguousarray(Xv, dtype=np.float32)
    yv = np.ascontiguousarray(yv, dtype=np.int32)
    ww = np.ascontiguousarray(ww, dtype=np.float64)
    D = np.ascontiguousarray(np.atleast_2d(deltas), dtype=np.float64)
    nv, din = Xv.shape
    assert ww.shape == (n_classes * (din + 1),) and D.shape[1] == ww.shape[0]
    out = np.empty(D.shape[0], dtype=np.float64)
    nt = np.empty(D.shape[0] + 1, dtype=np.int32)
    assert lib().oracle_roni_softmax(_ptr(Xv), nv, din, din, _ptr(yv), int(n_classes), _ptr(ww),
                                     _ptr(D), D.shape[0], D.shape[1], _ptr(out), _ptr(nt)) == 0
    return (out, nt) if near_ties else out


def roni_softmax_batches(Xv, yv, n_classes, ww, deltas, idx):
    """The reference's last-batch semantics (client.py:136-144): update j's
    `original` on the samples idx[j, 0] (model ww) and its `after` on idx[j, 1]
    (model ww + delta_j).  idx (n, 2, nb) int64.  Returns (scores (n,),
    near_ties (n, 2))."""
    Xv = np.ascontiguousarray(Xv, dtype=np.float32)
    yv = np.ascontiguousarray(yv, dtype=np.int32)
    ww = np.ascontiguousarray(ww, dtype=np.float64)
    D = np.ascontiguousarray(np.atleast_2d(deltas), dtype=np.float64)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    nv, din = Xv.shape
    n = D.shape[0]
    assert idx.ndim == 3 and idx.shape[:2] == (n, 2)
    nb = idx.shape[2]
    out = np.empty(n, dtype=np.float64)
    nt = np.empty((n, 2), dtype=np.int32)
    assert lib().oracle_roni_softmax_batches(_ptr(Xv), nv, din, din, _ptr(yv), int(n_classes),
                                             _ptr(ww), _ptr(D), n, D.shape[1], _ptr(idx), nb,
                                             _ptr(out), _ptr(nt)) == 0
    return out, nt
