"""Host-side mirror of the steps either side of the Multi-Krum verifier
(SURVEY.md §8(f) rows 2 and 3), on libbk.

  create_block(global_w, block_updates, stake_map)
        Honest.createBlock, DistSys/honest.go:346-381: GlobalW += Delta of
        every accepted update, in blockUpdates order (bk_aggregate), and the
        +-STAKE_UNIT stake bookkeeping (honest.go:46, :364-369; host logic).
  quantized_sum(deltas, idx, precision)
        updateFloatToInt (DistSys/kyber.go:698-710) of each accepted update,
        summed as the miners' share aggregation does (honest.go:401-409,
        442-502), and updateIntToFloat (kyber.go:745-757)
        (bk_quantized_sum_device).
  apply_noise(delta, noise)
        requestNoiseFromNoisers' average (DistSys/main.go:1606-1653) added
        to Delta (main.go:1524-1537), batched over updates
        (bk_noise_apply_device).

The arithmetic runs in libbk.so on the GPU (torch only moves buffers); there
is no CPU path.
"""
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from .krum import Engine, Update, default_engine

__all__ = ["STAKE_UNIT", "PRECISION", "create_block", "quantized_sum", "apply_noise"]

STAKE_UNIT = 5   # DistSys/honest.go:46
PRECISION = 4    # DistSys/main.go:45


def _engine(engine: Optional[Engine]) -> Engine:
    return engine if engine is not None else default_engine(0)


def create_block(global_w: np.ndarray, block_updates: Sequence[Update],
                 stake_map: Dict[int, int], engine: Optional[Engine] = None) -> np.ndarray:
    """honest.go:346-381 minus the chain append: returns the updated gradient
    (a new array, like mat.Row into updatedGradient) and updates stake_map in
    place.  Accepted updates are added in blockUpdates order."""
    out = np.array(global_w, dtype=np.float64, copy=True)
    d = out.shape[0]
    accepted: List[int] = []
    for i, u in enumerate(block_updates):
        their = stake_map.get(u.SourceID, 0)
        if u.Accepted:
            accepted.append(i)
            stake_map[u.SourceID] = their + STAKE_UNIT
        else:
            stake_map[u.SourceID] = their - STAKE_UNIT
    if not accepted:
        return out
    X = np.empty((len(block_updates), d), dtype=np.float64)
    for i, u in enumerate(block_updates):
        if u.Accepted:
            delta = np.asarray(u.Delta, dtype=np.float64)
            if delta.shape != (d,):
                raise ValueError("update %d: Delta has %s entries, gradient has %d"
                                 % (i, delta.shape, d))
            X[i] = delta
        else:
            X[i] = 0.0  # never read
    _engine(engine).aggregate(X, np.asarray(accepted, dtype=np.int64), out)
    return out


def quantized_sum(deltas, idx, precision: int = PRECISION, engine: Optional[Engine] = None):
    """(int64 sum, float64 sum) over rows idx of deltas (n x d), each row
    quantised as int64(x * 10^precision) (Go amd64 truncation)."""
    import torch
    eng = _engine(engine)
    X = np.ascontiguousarray(deltas)
    if X.dtype not in (np.float64, np.float32):
        X = X.astype(np.float64)
    n, d = X.shape
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    if idx.size and (idx.min() < 0 or idx.max() >= n):
        raise ValueError("idx out of range [0, %d)" % n)
    dev = torch.device("cuda", eng.device)
    tX = torch.from_numpy(X).to(dev)
    tI = torch.from_numpy(idx).to(dev)
    s = torch.empty(d, dtype=torch.int64, device=dev)
    sf = torch.empty(d, dtype=torch.float64, device=dev)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    dt = _lib.BK_F32 if X.dtype == np.float32 else _lib.BK_F64
    eng.quantized_sum_ptr(tX.data_ptr(), dt, n, d, d, tI.data_ptr(), len(idx), precision,
                          s.data_ptr(), sf.data_ptr())
    torch.cuda.synchronize(dev)
    return s.cpu().numpy(), sf.cpu().numpy()


def apply_noise(delta, noise, engine: Optional[Engine] = None) -> np.ndarray:
    """NoisedDelta for a batch: delta (n x d) or (d,), noise (n x k x d) or
    (k x d) -- noise vectors in arrival order."""
    import torch
    eng = _engine(engine)
    D = np.ascontiguousarray(delta, dtype=np.float64)
    N = np.ascontiguousarray(noise, dtype=np.float64)
    single = D.ndim == 1
    if single:
        D, N = D[None], N[None]
    n, d = D.shape
    if N.ndim != 3 or N.shape[0] != n or N.shape[2] != d:
        raise ValueError("noise must be (n, k, d) matching delta (n, d)")
    k = N.shape[1]
    dev = torch.device("cuda", eng.device)
    tD = torch.from_numpy(D).to(dev)
    tN = torch.from_numpy(N.reshape(n * k, d) if k else np.zeros((1, d))).to(dev)
    out = torch.empty_like(tD)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    eng.noise_apply_ptr(tD.data_ptr(), n, d, d, tN.data_ptr(), k, d, out.data_ptr(), d)
    torch.cuda.synchronize(dev)
    o = out.cpu().numpy()
    return o[0] if single else o
