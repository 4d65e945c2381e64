"""A/B builds of K1i8 (the int8-sliced Gram, bk_i8.hip) in ONE process on ONE GPU.

    python tools/ab_i8.py base=tools/ab/libbk_base.so new=biscotti_amd/libbk.so

Each build's context runs bk_gram_upper_device on the same device batch (config
E by default: 4,096 x 262,144 fp32 under BK_F32_I8; DT=f64 N=512 D=1048576 for
the headline batch under BK_F64_I8), interleaved REPS times; per build the
median of k_slice (slicing + bound), k_gram (k_gram_i8) and k_reduce, the int8
rate of k_gram over its 6 n(n+1)d digit-product ops, and whether the packed
upper equals the first build's bit for bit.
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import torch  # noqa: E402

from ab_libs import load  # noqa: E402
from biscotti_amd import _lib  # noqa: E402

KIDS = ("k_slice", "k_gram", "k_reduce")


def kid_of(lib, name):
    return _lib.KERNELS.index(name)


def run(lib, ctx, X, dt, n, d, U, reps):
    lib.bk_gram_upper_device(ctx, X, dt, n, d, d, U)
    lib.bk_synchronize(ctx)
    lib.bk_timing_enable(ctx, 1)
    for _ in range(reps):
        st = lib.bk_gram_upper_device(ctx, X, dt, n, d, d, U)
        assert st == 0, lib.bk_last_error()
    lib.bk_synchronize(ctx)
    out = {}
    for name in KIDS:
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        if lib.bk_timing_read(ctx, kid_of(lib, name), ctypes.byref(ms), ctypes.byref(cnt)) != 0:
            ms.value, cnt.value = float("nan"), 1
        out[name] = ms.value / max(cnt.value, 1)
    lib.bk_timing_enable(ctx, 0)
    return out


def main():
    f64 = os.environ.get("DT", "f32") == "f64"
    n = int(os.environ.get("N", 512 if f64 else 4096))
    d = int(os.environ.get("D", (1 << 20) if f64 else 262144))
    reps = int(os.environ.get("REPS", 5))
    rounds = int(os.environ.get("ROUNDS", 4))
    builds = []
    for a in sys.argv[1:]:
        label, path = a.split("=", 1)
        builds.append((label,) + load(path))
    dt = _lib.BK_F64 if f64 else _lib.BK_F32
    X = torch.empty((n, d), dtype=torch.float64 if f64 else torch.float32, device="cuda")
    lib0, ctx0 = builds[0][1], builds[0][2]
    lib0.bk_synth_fill_device(ctx0, X.data_ptr(), dt, n, d, d, 0, d, 1, n // 3, 0.01, 0.05, 1e-3, 0)
    lib0.bk_synchronize(ctx0)
    mode = int(os.environ.get("MODE", 3))  # 3: three digits (BK_F32_I8); 5: two (BK_F32_I8X2)
    for label, lib, ctx, env in builds:
        st = (lib.bk_set_f64_mode(ctx, mode) if f64 else lib.bk_set_f32_mode(ctx, mode))
        assert st == 0, lib.bk_last_error()
    ue = int(lib0.bk_upper_elems(n))
    Us = {b[0]: torch.empty(ue, dtype=torch.float64, device="cuda") for b in builds}
    res = {b[0]: [] for b in builds}
    for _ in range(rounds):
        for label, lib, ctx, env in builds:
            res[label].append(run(lib, ctx, X.data_ptr(), dt, n, d, Us[label].data_ptr(), reps))
    torch.cuda.synchronize()
    ref = Us[builds[0][0]]
    ops = (3 if mode == 5 else 6) * n * (n + 1) * d
    for label, v in res.items():
        med = {k: sorted(x[k] for x in v)[len(v) // 2] for k in KIDS}
        same = bool(torch.equal(Us[label], ref))
        print("%-8s n=%d d=%d %s  slice %.3f ms  gram %.3f ms (%.0f TOPS int8, %.3f of 4900)  "
              "reduce %.3f ms  total %.3f ms  upper==%s: %s" %
              (label, n, d, "f64" if f64 else "f32", med["k_slice"], med["k_gram"],
               ops / (med["k_gram"] * 1e-3) / 1e12, ops / (med["k_gram"] * 1e-3) / 4.9e15,
               med["k_reduce"], sum(med.values()), builds[0][0], same), flush=True)


if __name__ == "__main__":
    main()
