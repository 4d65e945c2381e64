"""Dimension-sharded Multi-Krum across the GPUs of one node (one process each).

SURVEY.md §8(e): the Gram matrix is additive over columns,
G = sum_g X[:, d_g] X[:, d_g]^T, so rank g owns a contiguous column shard d_g,
computes its packed partial Gram, and ONE exchange (RCCL all-reduce over xGMI,
inside libbk) gives every rank the full Gram.  Scores and selection are then
computed redundantly on every rank (microseconds) and each rank writes the
mean of its own columns, so no second collective is needed.

The reference has no such dimension (its verifiers are independent replicas,
DistSys/main.go:1680-1682); this is the MI355X build's own scale-out axis.

Host-side pieces here are backend-neutral so the CPU tests can drive the same
orchestration with gloo (tests/test_dist_gloo.py).
"""
import numpy as np

ALIGN = 8  # shard boundaries on 8-column (64 B fp64) multiples: keeps 16-B loads aligned


def shard_bounds(d, world, rank, align=ALIGN):
    """Contiguous column shard [c0, c0 + dl) of rank `rank` out of `world`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per = -(-d // world)
    per = -(-per // align) * align
    c0 = min(d, rank * per)
    c1 = min(d, c0 + per)
    return c0, c1 - c0


def all_shards(d, world, align=ALIGN):
    return [shard_bounds(d, world, r, align) for r in range(world)]


def upper_elems(n):
    """bk_upper_elems: the 64x64 upper sub-tiles + the trailing record {column
    count, columns accumulated on the fp32 MFMA, the int8-sliced Gram's absolute
    error bound, 0} (summed by the exchange with the tiles; the selection
    margin's d, unit roundoff and Gram error)."""
    T = (n + 63) // 64
    return T * (T + 1) // 2 * 4096 + 4


def pack_upper(G, d_cols, d_cols_f32=0):
    """Dense symmetric n x n -> the packed 64x64-sub-tile upper layout libbk
    exchanges (bk_upper_elems(n) doubles, sub-tiles (bi <= bj) row-major, then
    the column count d_cols the partial was taken over and how many of them
    were accumulated at fp32 unit roundoff).  d_cols is required: the margin's
    error bound grows with it, and a record with d_cols < 1 makes every
    selection a near tie (err_bound = +inf)."""
    if d_cols is None:
        raise ValueError("pack_upper needs the partial's column count")
    n = G.shape[0]
    T = (n + 63) // 64
    Gp = np.zeros((T * 64, T * 64))
    Gp[:n, :n] = G
    out = np.zeros((T * (T + 1) // 2, 64, 64))
    u = 0
    for bi in range(T):
        for bj in range(bi, T):
            out[u] = Gp[bi * 64:(bi + 1) * 64, bj * 64:(bj + 1) * 64]
            u += 1
    return np.concatenate([out.reshape(-1), [float(d_cols), float(d_cols_f32), 0.0, 0.0]])


def unpack_upper(U, n):
    """Inverse of pack_upper (upper sub-tiles; diagonal sub-tiles: i <= j used)."""
    T = (n + 63) // 64
    tiles = np.asarray(U)[:T * (T + 1) // 2 * 4096].reshape(-1, 64, 64)
    Gp = np.zeros((T * 64, T * 64))
    u = 0
    for bi in range(T):
        for bj in range(bi, T):
            t = tiles[u]
            if bi == bj:
                t = np.triu(t) + np.triu(t, 1).T
                Gp[bi * 64:(bi + 1) * 64, bj * 64:(bj + 1) * 64] = t
            else:
                Gp[bi * 64:(bi + 1) * 64, bj * 64:(bj + 1) * 64] = t
                Gp[bj * 64:(bj + 1) * 64, bi * 64:(bi + 1) * 64] = t.T
            u += 1
    return Gp[:n, :n]


def bootstrap_rccl(engine, rank, world, broadcast_bytes):
    """Create libbk's RCCL communicator.  `broadcast_bytes(b, src)` is any
    out-of-band broadcast (torch.distributed, gloo, MPI, a Go RPC...)."""
    from .krum import comm_unique_id
    uid = comm_unique_id() if rank == 0 else bytes(128)
    uid = broadcast_bytes(uid, 0)
    engine.comm_init(world, rank, uid)


def torch_broadcast_bytes(b, src=0):
    """Broadcast a short byte string with torch.distributed (any backend)."""
    import torch.distributed as dist
    obj = [bytes(b)]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


class ShardedKrum:
    """Host orchestration of one sharded Multi-Krum step.

    The three hooks are the product path's stages; tests on CPU replace them
    (gram_partial / finish with the oracle, exchange with gloo) to check the
    decomposition and the orchestration without a GPU.
    """

    def __init__(self, n, d, f, world, rank):
        self.n, self.d, self.f = n, d, f
        self.world, self.rank = world, rank
        self.c0, self.dl = shard_bounds(d, world, rank)

    def gram_partial(self, X_local):  # -> packed partial Gram (bk_gram_upper_device)
        raise NotImplementedError

    def exchange(self, U):  # -> summed packed Gram (RCCL all-reduce in libbk)
        raise NotImplementedError

    def finish(self, U, X_local):  # -> (sel, scores, mean_local) (bk_finish_device)
        raise NotImplementedError

    def step(self, X_local):
        U = self.gram_partial(X_local)
        U = self.exchange(U)
        return self.finish(U, X_local)
