"""Host-side mirror of Biscotti's RONI verifier, on libbk.

  roni(ww, delta)                 ML/code/logistic_validator.py:22-33 (the
                                  validation set is the module's, set once
                                  with set_validation -- the module body loads
                                  it at import, :6-7)
  RONIValidator                   Honest.verifyUpdate, DistSys/honest.go:598-629
    .verify_update(update)        Peer.VerifyUpdateRONI, DistSys/main.go:191-233:
                                  accept iff PRIV_PROB > 0 or score <= 0.02
    .scores(ww, deltas)           the batched form (one launch for n updates)

Everything runs through libbk.so on the GPU (bk_roni_set_validation / bk_roni);
there is no CPU path.
"""
from typing import Optional, Sequence

import numpy as np

from ._lib import check, lib
from .krum import Engine, Update, default_engine

__all__ = ["RONI_THRESHOLD", "RONIValidator", "SoftmaxRONIValidator", "set_validation", "roni"]

RONI_THRESHOLD = 0.02  # main.go:213


class RONIValidator:
    """One validation set resident on one GPU (bk_roni_set_validation)."""

    def __init__(self, Xvalid, yvalid, engine: Optional[Engine] = None, priv_prob: float = 0.0):
        self._engine = engine if engine is not None else default_engine(0)
        X = np.ascontiguousarray(Xvalid, dtype=np.float64)
        y = np.ascontiguousarray(yvalid, dtype=np.float64)
        if X.ndim != 2 or y.shape != (X.shape[0],):
            raise ValueError("Xvalid must be (nv, d) and yvalid (nv,)")
        self.nv, self.d = X.shape
        self.priv_prob = priv_prob  # PRIV_PROB > 0 accepts every update (main.go:205-211)
        check(lib().bk_roni_set_validation(self._engine.ctx, X.ctypes.data, self.nv, self.d,
                                           self.d, y.ctypes.data))

    def scores(self, ww, deltas) -> np.ndarray:
        ww = np.ascontiguousarray(ww, dtype=np.float64)
        D = np.ascontiguousarray(np.atleast_2d(deltas), dtype=np.float64)
        if ww.shape != (self.d,) or D.shape[1] != self.d:
            raise ValueError("ww must be (d,) and deltas (n, d) with d = %d" % self.d)
        out = np.empty(D.shape[0], dtype=np.float64)
        check(lib().bk_roni(self._engine.ctx, ww.ctypes.data, D.ctypes.data, D.shape[0], self.d,
                            self.d, out.ctypes.data))
        return out

    def roni(self, ww, delta) -> float:
        return float(self.scores(ww, np.asarray(delta)[None])[0])

    def verify_update(self, update: Update, latest_gradient) -> bool:
        """True = accept (sign), False = reject (updateError)."""
        score = self.roni(latest_gradient, update.NoisedDelta)
        if self.priv_prob > 0:
            return True
        return not (score > RONI_THRESHOLD)

    def verify_updates(self, updates: Sequence[Update], latest_gradient) -> np.ndarray:
        """The batched form: one launch scores every update."""
        sc = self.scores(latest_gradient, np.stack([u.NoisedDelta for u in updates]))
        if self.priv_prob > 0:
            return np.ones(len(updates), dtype=bool)
        return ~(sc > RONI_THRESHOLD)


class SoftmaxRONIValidator(RONIValidator):
    """The torch-path verifier (ML/Pytorch/client_obj.py:100-112: the mnist /
    lfw softmax models): err = 1 - accuracy of argmax(x W^T + b)
    (client.py:136-144), the flat weights [W (C x d_in), b (C)] rounded to fp32
    as SoftmaxModel.reshape does.  The client's training shard is resident on
    one GPU (bk_roni_softmax_set_validation).

    Which samples: getTrainErr walks the SHUFFLED trainloader (client.py:20)
    and returns the error of its LAST mini-batch, so `original` and `after`
    are each measured on a fresh random last batch of batch_size samples (10
    in Biscotti, DistSys/honest.go:47).  This mirror draws those batches as the
    DataLoader does -- a permutation per pass, the last batch its tail of
    nv % batch_size (or batch_size) samples -- from its own seeded generator,
    and scores them with bk_roni_softmax_batches.  batch_size=None (or >= nv)
    scores every evaluation over the whole set (bk_roni_softmax).

    After each call, last_near_ties holds the per-evaluation near-tie counts
    (bk.h: where torch's fp32 argmax may differ from this one) and last_idx
    the (n, 2, nb) sample indices it scored (None for whole-set scores): the
    reference's scores are random draws (client.py:136-144), so a decision is
    reproduced by passing last_idx back as idx, or by a fixed seed.  A
    validator built with seed=None draws from fresh OS entropy each run."""

    def __init__(self, Xvalid, yvalid, n_classes, engine: Optional[Engine] = None,
                 priv_prob: float = 0.0, batch_size: Optional[int] = 10, seed=None):
        self._engine = engine if engine is not None else default_engine(0)
        X = np.ascontiguousarray(Xvalid, dtype=np.float32)
        y = np.ascontiguousarray(yvalid, dtype=np.int32)
        if X.ndim != 2 or y.shape != (X.shape[0],):
            raise ValueError("Xvalid must be (nv, d_in) and yvalid (nv,)")
        self.nv, self.d_in = X.shape
        self.n_classes = int(n_classes)
        self.d = self.n_classes * (self.d_in + 1)
        self.priv_prob = priv_prob
        self.batch_size = None if batch_size is None or batch_size >= self.nv else int(batch_size)
        if self.batch_size is not None and self.batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        self._rng = np.random.default_rng(seed)
        self.last_near_ties = None
        self.last_idx = None
        check(lib().bk_roni_softmax_set_validation(self._engine.ctx, X.ctypes.data, self.nv,
                                                   self.d_in, self.d_in, y.ctypes.data,
                                                   self.n_classes))

    def last_batch(self) -> np.ndarray:
        """One shuffled pass's last mini-batch (DataLoader(shuffle=True))."""
        perm = self._rng.permutation(self.nv)
        nb = self.nv % self.batch_size or self.batch_size
        return perm[self.nv - nb:]

    def draw_batches(self, n) -> np.ndarray:
        """(n, 2, nb) indices: per update, the batch `original` then the batch
        `after` is scored on, in the reference's call order."""
        return np.array([[self.last_batch(), self.last_batch()] for _ in range(n)], dtype=np.int64)

    def scores(self, ww, deltas, idx=None) -> np.ndarray:
        ww = np.ascontiguousarray(ww, dtype=np.float64)
        D = np.ascontiguousarray(np.atleast_2d(deltas), dtype=np.float64)
        if ww.shape != (self.d,) or D.shape[1] != self.d:
            raise ValueError("ww must be (d,) and deltas (n, d) with d = %d" % self.d)
        n = D.shape[0]
        out = np.empty(n, dtype=np.float64)
        if idx is None and self.batch_size is None:
            nt = np.empty(n + 1, dtype=np.int32)
            check(lib().bk_roni_softmax(self._engine.ctx, ww.ctypes.data, D.ctypes.data, n,
                                        self.d, out.ctypes.data, nt.ctypes.data))
            self.last_near_ties = nt
            self.last_idx = None
            return out
        idx = self.draw_batches(n) if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        self.last_idx = idx
        if idx.ndim != 3 or idx.shape[:2] != (n, 2):
            raise ValueError("idx must be (n, 2, nb)")
        nt = np.empty((n, 2), dtype=np.int32)
        check(lib().bk_roni_softmax_batches(self._engine.ctx, ww.ctypes.data, D.ctypes.data, n,
                                            self.d, idx.ctypes.data, idx.shape[2],
                                            out.ctypes.data, nt.ctypes.data))
        self.last_near_ties = nt
        return out


_validator: Optional[RONIValidator] = None


def set_validation(Xvalid, yvalid, engine: Optional[Engine] = None):
    """The module-level validation set (logistic_validator.py:6-7)."""
    global _validator
    _validator = RONIValidator(Xvalid, yvalid, engine)
    return _validator


def roni(ww, delta) -> float:
    """logistic_validator.py:22-33 against the set given to set_validation."""
    if _validator is None:
        raise RuntimeError("call set_validation(Xvalid, yvalid) first (the module loads it)")
    return _validator.roni(ww, delta)
