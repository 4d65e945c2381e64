"""numpy restatement of the synthetic-input spec (DESIGN.md "Synthetic inputs").

Test infrastructure: used by gen_goldens.py to build the exact inputs the
reference ``krum`` is run on, and by the CPU tests to check that the C oracle
generator (oracle/krum_oracle.c) and the GPU generator
(biscotti_amd/csrc/bk_synth.h) produce the same bits.

All arithmetic is uint64 wrap-around hashing (SplitMix64) plus IEEE add/mul
with no fused operations, so numpy, gcc and hipcc agree bit-for-bit.
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GAMMA = np.uint64(0x9E3779B97F4A7C15)
C1 = np.uint64(0xBF58476D1CE4E5B9)
C2 = np.uint64(0x94D049BB133111EB)
STREAM_MUL = np.uint64(0xD1B54A32D192ED03)
SQRT3 = 1.7320508075688772
FP32ROUND = 1


def sm64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + GAMMA
        x = (x ^ (x >> np.uint64(30))) * C1
        x = (x ^ (x >> np.uint64(27))) * C2
        return x ^ (x >> np.uint64(31))


def stream_base(seed, stream):
    with np.errstate(over="ignore"):
        return sm64(sm64(np.uint64(seed)) ^ (np.uint64(stream) * STREAM_MUL))


def u01(h):
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def gauss(base, idx):
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        c = base + np.uint64(4) * idx
        u0 = u01(sm64(c))
        u1 = u01(sm64(c + np.uint64(1)))
        u2 = u01(sm64(c + np.uint64(2)))
        u3 = u01(sm64(c + np.uint64(3)))
    return (((u0 + u1) + (u2 + u3)) - 2.0) * SQRT3


def synth_perm(seed, n):
    b = stream_base(seed, 3)
    perm = list(range(n))
    for i in range(n - 1, 0, -1):
        with np.errstate(over="ignore"):
            h = int(sm64(b + np.uint64(i)))
        j = h % (i + 1)
        perm[i], perm[j] = perm[j], perm[i]
    return np.array(perm, dtype=np.int64)


def synth(n, d, seed, nbyz, mu_scale=0.01, byz_scale=0.05, sigma=1e-3, flags=0,
          dtype=np.float64, c0=0, dl=None, d_total=None, row_chunk=64):
    """Rows [0,n) x columns [c0, c0+dl) of the n x d_total synthetic batch."""
    if dl is None:
        dl = d - c0
    if d_total is None:
        d_total = d
    perm = synth_perm(seed, n)
    b0, b1, b2, b4 = (stream_base(seed, s) for s in (0, 1, 2, 4))
    cols = np.arange(c0, c0 + dl, dtype=np.uint64)
    mu = mu_scale * gauss(b0, cols)
    byz_base = mu + byz_scale * gauss(b1, cols)
    out = np.empty((n, dl), dtype=dtype)
    for p0 in range(0, n, row_chunk):
        p1 = min(n, p0 + row_chunk)
        rows = perm[p0:p1]
        e = rows.astype(np.uint64)[:, None] * np.uint64(d_total) + cols[None, :]
        nz = sigma * gauss(b2, e)
        isbyz = (rows >= n - nbyz)[:, None]
        x = np.where(isbyz, byz_base[None, :], mu[None, :]) + nz
        if flags & FP32ROUND:
            x = x.astype(np.float32).astype(np.float64) + 1e-6 * gauss(b4, e)
        out[p0:p1] = x.astype(dtype)
    return out
