"""Host-side mirror of Biscotti's Multi-Krum verifier interface, on libbk.

Reference surface kept (same names, argument meaning and error behaviour):

  krum(deltas, clip)              ML/code/logistic_validator.py:36-49
                                  (== ML/Pytorch/client_obj.py:114-127)
  get_krum_scores(X, groupsize)   ML/code/logistic_validator.py:54-65
  KRUMValidator                   DistSys/krum.go:22-29
    .initialize()                 krum.go:31-44   (binds the engine instead of pyKRUMFunc)
    .check_if_accepted(peer_id)   krum.go:47-73
    .compute_scores()             krum.go:77-98
    .get_top_krum_index(deltas)   krum.go:100-166 (the go-python call this engine replaces)
    .flush_collected_updates()    krum.go:169-176
  Update                          DistSys/update.go:13-22

Differences a caller can observe, all documented in DESIGN.md:
  * the selected indices come back ascending (a set; numpy returns
    argpartition order, and the only consumer tests membership);
  * ties at the selection boundary resolve to the lower index;
  * clip = 0 raises ValueError, as np.argpartition does in the reference.

Everything runs through libbk.so on the GPU; there is no CPU path.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import ctypes
import numpy as np

from . import _lib
from ._lib import check, lib

__all__ = ["Engine", "krum", "get_krum_scores", "krum_mean", "KRUMValidator", "Update",
           "default_engine"]


def _p(x):
    return ctypes.c_void_p(x) if x is not None else None


def _as_rows(X):
    X = np.asarray(X)
    if X.dtype not in (np.float64, np.float32):
        X = X.astype(np.float64)
    if X.ndim != 2:
        raise ValueError("deltas must be 2-D (n updates x d)")
    if X.strides[1] != X.itemsize or X.strides[0] % X.itemsize:
        X = np.ascontiguousarray(X)
    return X


class GroupEngine:
    """One process driving G GPUs (bk_group_*): the Go verifier's multi-GPU
    form.  Each device copies its column shard of the host batch over its own
    PCIe link; the partial Grams are summed (RCCL all-reduce, RCCL all-gather
    + fixed-order sum, or a fixed-order sum through pinned host memory); every
    device selects identically and writes the mean of its columns."""

    def __init__(self, devices, mode=_lib.BK_GROUP_ALLREDUCE):
        devices = [int(x) for x in devices]
        arr = (ctypes.c_int * len(devices))(*devices)
        self._g = ctypes.c_void_p()
        check(lib().bk_group_create(ctypes.byref(self._g), len(devices), arr, int(mode)))
        self.devices = devices

    def close(self):
        if self._g:
            lib().bk_group_destroy(self._g)
            self._g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def size(self):
        return lib().bk_group_size(self._g)

    def ctx(self, r):
        return lib().bk_group_ctx(self._g, int(r))

    def multikrum(self, X, f, want_scores=True, want_mean=True, pinned=False):
        """bk_group_multikrum on a host batch: (sel ascending, scores, mean)."""
        X = _as_rows(X)
        n, d = X.shape
        f = int(f)
        check(lib().bk_check_args(n, d, f))
        m = n - f
        sel = np.empty(m, dtype=np.int64)
        mo = ctypes.c_int64(0)
        sc = np.empty(n, dtype=np.float64) if want_scores else None
        mean = np.empty(d, dtype=np.float64) if want_mean else None
        dt = _lib.BK_F32 if X.dtype == np.float32 else _lib.BK_F64
        check(lib().bk_group_multikrum(self._g, X.ctypes.data,
                                       _lib.BK_HOST_PINNED if pinned else _lib.BK_HOST, dt, n, d,
                                       X.strides[0] // X.itemsize, f, sel.ctypes.data,
                                       ctypes.addressof(mo),
                                       sc.ctypes.data if sc is not None else None,
                                       mean.ctypes.data if mean is not None else None))
        assert mo.value == m
        return sel, sc, mean


class Engine:
    """One libbk context (bk_ctx) bound to one GPU."""

    def __init__(self, device=0):
        self._ctx = ctypes.c_void_p()
        check(lib().bk_create(ctypes.byref(self._ctx), int(device)))
        self.device = int(device)

    def close(self):
        if self._ctx:
            lib().bk_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    # ---- host entry (bk_multikrum): numpy in, numpy out -----------------
    def multikrum(self, X, f, want_scores=True, want_mean=True):
        X = np.asarray(X)
        if X.dtype not in (np.float64, np.float32):
            X = X.astype(np.float64)
        if X.ndim != 2:
            raise ValueError("deltas must be 2-D (n updates x d)")
        if X.strides[1] != X.itemsize or X.strides[0] % X.itemsize:
            X = np.ascontiguousarray(X)
        n, d = X.shape
        ld = X.strides[0] // X.itemsize
        f = int(f)
        check(lib().bk_check_args(n, d, f))
        m = n - f
        sel = np.empty(m, dtype=np.int64)
        mo = ctypes.c_int64(0)
        sc = np.empty(n, dtype=np.float64) if want_scores else None
        mean = np.empty(d, dtype=np.float64) if want_mean else None
        dt = _lib.BK_F32 if X.dtype == np.float32 else _lib.BK_F64
        check(lib().bk_multikrum(self._ctx, X.ctypes.data, _lib.BK_HOST, dt, n, d, ld, f,
                                 sel.ctypes.data, ctypes.addressof(mo),
                                 sc.ctypes.data if sc is not None else None,
                                 mean.ctypes.data if mean is not None else None))
        assert mo.value == m
        return sel, sc, mean

    # ---- row-fed host entry (bk_multikrum_rows): n separate host rows, ---
    #      as the Go verifier holds them (deltas [][]float64, krum.go:100-166)
    def multikrum_rows(self, rows, f, want_scores=True, want_mean=True):
        """rows: a sequence of n 1-D arrays (all float64 or all float32, each d
        long, each contiguous); they are packed on libbk's host threads, not
        here.  Returns (sel, scores, mean) as multikrum."""
        rows = list(rows)
        n = len(rows)
        if n == 0:
            raise ValueError("no rows")
        dt = np.asarray(rows[0]).dtype
        if dt not in (np.float64, np.float32):
            raise ValueError("rows must be float64 or float32")
        keep = []
        for r in rows:
            a = np.asarray(r)
            if a.dtype != dt or a.ndim != 1:
                raise ValueError("every row must be a 1-D array of the first row's dtype")
            keep.append(a if a.flags.c_contiguous else np.ascontiguousarray(a))
        d = keep[0].shape[0]
        if any(a.shape[0] != d for a in keep):
            raise ValueError("ragged rows")
        f = int(f)
        check(lib().bk_check_args(n, d, f))
        m = n - f
        ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in keep])
        sel = np.empty(m, dtype=np.int64)
        mo = ctypes.c_int64(0)
        sc = np.empty(n, dtype=np.float64) if want_scores else None
        mean = np.empty(d, dtype=np.float64) if want_mean else None
        check(lib().bk_multikrum_rows(self._ctx, ptrs, _lib.BK_F32 if dt == np.float32 else
                                      _lib.BK_F64, n, d, f, sel.ctypes.data,
                                      ctypes.addressof(mo),
                                      sc.ctypes.data if sc is not None else None,
                                      mean.ctypes.data if mean is not None else None))
        assert mo.value == m
        return sel, sc, mean

    def multikrum_rows_ptr(self, row_ptrs, dtype, n, d, f, sel_ptr, scores_ptr=None,
                           mean_ptr=None):
        """Raw host row pointers (a ctypes c_void_p array); host outputs."""
        mo = ctypes.c_int64(0)
        check(lib().bk_multikrum_rows(self._ctx, row_ptrs, dtype, n, d, f, _p(sel_ptr),
                                      ctypes.addressof(mo), _p(scores_ptr), _p(mean_ptr)))
        return mo.value

    def set_host_threads(self, threads):
        check(lib().bk_set_host_threads(self._ctx, int(threads)))

    # ---- host entry with the noise applied in the H2D staging -----------
    #      (bk_multikrum_noised) -------------------
    def multikrum_noised(self, delta, noise, f, want_scores=True, want_mean=True,
                         want_noised=False):
        """Multi-Krum of NoisedDelta = delta + mean of the k noise vectors
        (main.go:1524-1537, 1606-1653) with the noise added on the device as
        the rows land.  delta (n, d) fp64; noise (n, k, d) fp64, k >= 0 (k = 0:
        no noisers, NoisedDelta = Delta).  Returns (sel, scores, mean, noised)."""
        D = np.asarray(delta, dtype=np.float64)
        if D.ndim != 2:
            raise ValueError("delta must be 2-D (n updates x d)")
        if D.strides[1] != 8 or D.strides[0] % 8:
            D = np.ascontiguousarray(D)
        n, d = D.shape
        N = np.ascontiguousarray(noise, dtype=np.float64)
        if N.ndim != 3 or N.shape[0] != n or (N.shape[1] > 0 and N.shape[2] != d):
            raise ValueError("noise must be (n, k, d) matching delta (n, d)")
        k = N.shape[1]
        f = int(f)
        check(lib().bk_check_args(n, d, f))
        m = n - f
        sel = np.empty(m, dtype=np.int64)
        mo = ctypes.c_int64(0)
        sc = np.empty(n, dtype=np.float64) if want_scores else None
        mean = np.empty(d, dtype=np.float64) if want_mean else None
        out = np.empty((n, d), dtype=np.float64) if want_noised else None
        check(lib().bk_multikrum_noised(self._ctx, D.ctypes.data, D.strides[0] // 8,
                                        N.ctypes.data if k else None, k, d, _lib.BK_HOST, n, d,
                                        f, sel.ctypes.data, ctypes.addressof(mo),
                                        sc.ctypes.data if sc is not None else None,
                                        mean.ctypes.data if mean is not None else None,
                                        out.ctypes.data if out is not None else None, d))
        assert mo.value == m
        return sel, sc, mean, out

    def multikrum_noised_ptr(self, delta_ptr, ld, noise_ptr, k, noise_ld, where, n, d, f,
                             sel_ptr, scores_ptr=None, mean_ptr=None, noised_ptr=None,
                             out_ld=0):
        """Raw host pointers (e.g. pinned torch tensors); outputs are host pointers."""
        mo = ctypes.c_int64(0)
        check(lib().bk_multikrum_noised(self._ctx, _p(delta_ptr), ld, _p(noise_ptr), k, noise_ld,
                                        where, n, d, f, _p(sel_ptr), ctypes.addressof(mo),
                                        _p(scores_ptr), _p(mean_ptr), _p(noised_ptr),
                                        out_ld or d))
        return mo.value

    # ---- device entry (bk_multikrum_device): raw device pointers --------
    def multikrum_device_ptr(self, x_ptr, dtype, n, d, ld, f, sel_ptr, scores_ptr=None,
                             mean_ptr=None):
        check(lib().bk_multikrum_device(self._ctx, _p(x_ptr), dtype, n, d, ld, f, _p(sel_ptr),
                                        _p(scores_ptr), _p(mean_ptr)))

    def multikrum_sharded_ptr(self, x_ptr, dtype, n, d_local, ld, f, sel_ptr, scores_ptr=None,
                              mean_ptr=None):
        check(lib().bk_multikrum_sharded_device(self._ctx, _p(x_ptr), dtype, n, d_local, ld, f,
                                                _p(sel_ptr), _p(scores_ptr), _p(mean_ptr)))

    # ---- SURVEY §8(f) rows 2-3 (bk_aggregate*, bk_quantized_sum_device,
    #      bk_noise_apply_device) --------------------------------------------
    def aggregate(self, X, idx, global_w):
        """global_w += X[idx[0]] + X[idx[1]] + ... in place (host arrays; bk_aggregate)."""
        X = np.asarray(X)
        if X.dtype not in (np.float64, np.float32):
            X = X.astype(np.float64)
        if X.strides[1] != X.itemsize or X.strides[0] % X.itemsize:
            X = np.ascontiguousarray(X)
        n, d = X.shape
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        if global_w.dtype != np.float64 or not global_w.flags.c_contiguous or global_w.shape != (d,):
            raise ValueError("global_w must be a C-contiguous float64 vector of length d")
        dt = _lib.BK_F32 if X.dtype == np.float32 else _lib.BK_F64
        check(lib().bk_aggregate(self._ctx, X.ctypes.data, _lib.BK_HOST, dt, n, d,
                                 X.strides[0] // X.itemsize, idx.ctypes.data, len(idx),
                                 global_w.ctypes.data))
        return global_w

    def aggregate_device_ptr(self, x_ptr, dtype, n, d, ld, idx_ptr, m, global_ptr):
        check(lib().bk_aggregate_device(self._ctx, _p(x_ptr), dtype, n, d, ld, _p(idx_ptr), m,
                                        _p(global_ptr)))

    def quantized_sum_ptr(self, x_ptr, dtype, n, d, ld, idx_ptr, m, precision, sum_ptr,
                          sumf_ptr=None):
        check(lib().bk_quantized_sum_device(self._ctx, _p(x_ptr), dtype, n, d, ld, _p(idx_ptr), m,
                                            int(precision), _p(sum_ptr), _p(sumf_ptr)))

    def noise_apply_ptr(self, delta_ptr, n, d, ld, noise_ptr, k, noise_ld, out_ptr, out_ld):
        check(lib().bk_noise_apply_device(self._ctx, _p(delta_ptr), n, d, ld, _p(noise_ptr), k,
                                          noise_ld, _p(out_ptr), out_ld))

    def gram_upper_ptr(self, x_ptr, dtype, n, d, ld, upper_ptr):
        check(lib().bk_gram_upper_device(self._ctx, _p(x_ptr), dtype, n, d, ld, _p(upper_ptr)))

    def finish_ptr(self, upper_ptr, x_ptr, dtype, n, d, ld, f, sel_ptr, scores_ptr=None,
                   mean_ptr=None):
        check(lib().bk_finish_device(self._ctx, _p(upper_ptr), _p(x_ptr), dtype, n, d, ld, f,
                                     _p(sel_ptr), _p(scores_ptr), _p(mean_ptr)))

    def synth_fill_ptr(self, x_ptr, dtype, n, d_local, ld, c0, d_total, seed, nbyz,
                       mu_scale=0.01, byz_scale=0.05, sigma=1e-3, flags=0):
        check(lib().bk_synth_fill_device(self._ctx, _p(x_ptr), dtype, n, d_local, ld, c0, d_total,
                                         seed, nbyz, mu_scale, byz_scale, sigma, flags))

    # ---- plumbing ------------------------------------------------------
    def set_stream(self, stream_handle):
        check(lib().bk_set_stream(self._ctx, _p(stream_handle)))

    def stream(self):
        return lib().bk_get_stream(self._ctx)

    def synchronize(self):
        check(lib().bk_synchronize(self._ctx))

    def comm_init(self, nranks, rank, uid_bytes):
        buf = ctypes.create_string_buffer(bytes(uid_bytes), _lib.BK_UNIQUE_ID_BYTES)
        check(lib().bk_comm_init(self._ctx, int(nranks), int(rank), buf))

    def comm_set_mode(self, mode):
        """0 (or False): all-reduce; 1 (or True): deterministic all-gather +
        rank-order sum; 2: all-reduce overlapped with the Gram (bk.h)."""
        check(lib().bk_comm_set_mode(self._ctx, int(mode)))

    def timing_enable(self, on=True):
        check(lib().bk_timing_enable(self._ctx, 1 if on else 0))

    # ---- selection margin (bk_selection_margin): where the selection may
    #      legitimately differ from numpy's (logistic_validator.py:45,59-63) --
    def selection_margin(self):
        """{gap, err_bound, near_tie, M, s_lo, s_hi, d, k} of the last call on
        this context; near_tie False proves the reference selects the same set."""
        rec = (ctypes.c_double * 8)()
        check(lib().bk_selection_margin_record(self._ctx, rec))
        keys = ("gap", "err_bound", "near_tie", "M", "s_lo", "s_hi", "d", "k")
        out = dict(zip(keys, (float(x) for x in rec)))
        out["near_tie"] = bool(out["near_tie"])
        out["d"] = int(out["d"])
        out["k"] = int(out["k"])
        return out

    def set_small_path(self, on=True):
        """n <= 128: the one-launch k_small path (default) or the general chain."""
        check(lib().bk_set_small_path(self._ctx, 1 if on else 0))

    def certified_reruns(self):
        return int(lib().bk_certified_reruns(self._ctx))

    def comm_size(self):
        nr, rk = ctypes.c_int(0), ctypes.c_int(0)
        check(lib().bk_comm_size(self._ctx, ctypes.byref(nr), ctypes.byref(rk)))
        return nr.value, rk.value

    def comm_stats(self):
        ex, by = ctypes.c_int64(0), ctypes.c_double(0)
        check(lib().bk_comm_stats(self._ctx, ctypes.byref(ex), ctypes.byref(by)))
        return ex.value, by.value

    def set_f32_mode(self, mode):
        """_lib.BK_F32_EXACT (fp32 rows widened onto the fp64 MFMA, default),
        _lib.BK_F32_MFMA (the fp32 MFMA, fp32 accumulation per K1 segment),
        _lib.BK_F32_CERTIFIED (the fp32 MFMA, re-run exactly on a near tie),
        _lib.BK_F32_I8 / _lib.BK_F32_I8_CERTIFIED (the Gram from exact int8
        digit slices, K1i8: three digits, six products), _lib.BK_F32_I8X2 /
        _lib.BK_F32_I8X2_CERTIFIED (two digits, three products)."""
        check(lib().bk_set_f32_mode(self._ctx, int(mode)))

    def set_f64_mode(self, mode):
        """fp64 rows: BK_F64_EXACT (the fp64 MFMA), BK_F64_I8 (the Gram from exact
        int8 digit slices, error bound in the margin) or BK_F64_I8_CERTIFIED
        (exact re-run on a near tie); BK_F64_I8X2 / BK_F64_I8X2_CERTIFIED the
        two-digit slicing."""
        check(lib().bk_set_f64_mode(self._ctx, int(mode)))

    def graph_enable(self, on=True):
        """Replay multikrum_device_ptr calls as hipGraphs (bk_graph_enable)."""
        check(lib().bk_graph_enable(self._ctx, 1 if on else 0))

    def timing_select(self, kernels):
        """Time only these kernels (names from _lib.KERNELS)."""
        mask = 0
        for k in kernels:
            mask |= 1 << _lib.K[k]
        check(lib().bk_timing_select(self._ctx, mask))

    def timing_stride(self, every):
        """Record a timed kernel's events on every `every`-th launch (bk_timing_stride)."""
        check(lib().bk_timing_stride(self._ctx, int(every)))

    def timing_read(self):
        out = {}
        for i, name in enumerate(_lib.KERNELS):
            ms = ctypes.c_double(0)
            cnt = ctypes.c_int64(0)
            check(lib().bk_timing_read(self._ctx, i, ctypes.byref(ms), ctypes.byref(cnt)))
            if cnt.value:
                out[name] = {"total_ms": ms.value, "count": cnt.value,
                             "avg_ms": ms.value / cnt.value}
        return out

    def plan(self, n, d):
        v = [ctypes.c_int64(0) for _ in range(4)]
        check(lib().bk_plan(self._ctx, n, d, *[ctypes.byref(x) for x in v]))
        return dict(zip(("S", "kc", "ntile", "nwg"), (x.value for x in v)))


def comm_unique_id():
    buf = ctypes.create_string_buffer(_lib.BK_UNIQUE_ID_BYTES)
    check(lib().bk_comm_unique_id(buf))
    return buf.raw


_default = {}


def default_engine(device=0):
    if device not in _default:
        _default[device] = Engine(device)
    return _default[device]


def _as_matrix(deltas):
    # logistic_validator.py:41 -- deltas = np.array(deltas)
    X = np.asarray(deltas)
    if X.dtype not in (np.float64, np.float32):
        X = np.array(deltas, dtype=np.float64)
    return X


def krum(deltas, clip, engine: Optional[Engine] = None):
    """Indices of the n - clip updates with the lowest Krum scores.

    Mirrors ``krum(deltas, clip)`` (logistic_validator.py:36-49); the result is
    the same index set, returned ascending.
    """
    X = _as_matrix(deltas)
    n = len(X)
    if clip < 1 or clip >= n:
        # np.argpartition(scores, n - clip) raises for kth == n (clip == 0)
        raise ValueError("kth(=%d) out of bounds (%d)" % (n - clip, n))
    sel, _, _ = (engine or default_engine()).multikrum(X, clip, want_scores=False,
                                                       want_mean=False)
    return sel


def krum_mean(deltas, clip, engine: Optional[Engine] = None):
    """(selected indices, mean of the selected deltas): the aggregate the
    reference leaves commented out at logistic_validator.py:51."""
    X = _as_matrix(deltas)
    n = len(X)
    if clip < 1 or clip >= n:
        raise ValueError("kth(=%d) out of bounds (%d)" % (n - clip, n))
    sel, _, mean = (engine or default_engine()).multikrum(X, clip, want_scores=False,
                                                          want_mean=True)
    return sel, mean


def get_krum_scores(X, groupsize, engine: Optional[Engine] = None):
    """Krum score of every row: sum of its groupsize-2 smallest distances to
    the others (logistic_validator.py:54-65).  groupsize = n - clip."""
    X = _as_matrix(X)
    n = len(X)
    f = n - int(groupsize)
    if f < 1 or f >= n:
        raise ValueError("groupsize must satisfy 1 <= n - groupsize < n")
    _, sc, _ = (engine or default_engine()).multikrum(X, f, want_scores=True, want_mean=False)
    return sc


@dataclass
class Update:
    """DistSys/update.go:13-22 (the fields the verifier path reads)."""
    SourceID: int
    Iteration: int = 0
    Delta: Optional[np.ndarray] = None
    Commitment: bytes = b""
    Noise: Optional[np.ndarray] = None
    NoisedDelta: Optional[np.ndarray] = None
    Accepted: bool = False
    SignatureList: List[bytes] = field(default_factory=list)


class KRUMValidator:
    """DistSys/krum.go:22-29, with getTopKRUMIndex running on libbk."""

    def __init__(self, num_adversaries=0.5, engine: Optional[Engine] = None, device=0):
        self.UpdateList: List[Update] = []
        self.AcceptedList: List[int] = []
        self.NumAdversaries = num_adversaries  # fixed at 0.5 (main.go:783)
        self._engine = engine
        self._device = device

    def initialize(self):
        # krum.go:31-44 bound pyKRUMFunc; here: create the engine context
        if self._engine is None:
            self._engine = default_engine(self._device)
        return self

    def check_if_accepted(self, peer_id):
        # krum.go:47-73 (the isPoisoning bypass at :51-58 is dead code: the
        # global is never set, main.go:843 declares a local)
        return any(self.UpdateList[i].SourceID == peer_id for i in self.AcceptedList)

    def compute_scores(self):
        # krum.go:77-98
        running = [u.NoisedDelta for u in self.UpdateList]
        self.AcceptedList = self.get_top_krum_index(running)

    def get_top_krum_index(self, deltas) -> List[int]:
        # krum.go:100-166: adversaryCount := int(NumAdversaries * float64(n))
        n = len(deltas)
        clip = int(self.NumAdversaries * float(n))
        if self._engine is None:
            self.initialize()
        # the rows go to libbk as they are (bk_multikrum_rows: packed on its
        # host threads into pinned memory, as the cgo shim hands Go's slices)
        rows = [np.asarray(r, dtype=np.float64) for r in deltas]
        sel, _, _ = self._engine.multikrum_rows(rows, clip, want_scores=False, want_mean=False)
        return [int(i) for i in sel]

    def flush_collected_updates(self, collecting_updates=False):
        # krum.go:169-176
        if not collecting_updates:
            self.UpdateList = []
            self.AcceptedList = []
