"""A/B two (or more) builds of libbk.so in ONE process on ONE GPU.

Boxes differ by several percent, so kernel changes are compared by loading
each build side by side (RTLD_LOCAL, separate code objects) and timing K1
interleaved on the same device buffer:

    python tools/ab_libs.py base=/path/libbk_base.so new=biscotti_amd/libbk.so \
        nosum=biscotti_amd/libbk.so,BK_CSUM=0

A ",KEY=VAL" suffix sets that env var while the build's context is created
(the context reads BK_* knobs at bk_create).  Env: N, D, REPS, and F: with F
set, time the whole bk_multikrum_device step and report K1 and K4 (k_mean).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd import _lib  # noqa: E402


def load(spec):
    path, *kv = spec.split(",")
    env = dict(x.split("=", 1) for x in kv)
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    ctx = ctypes.c_void_p()
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    st = lib.bk_create(ctypes.byref(ctx), 0)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    if st != 0:
        raise RuntimeError("%s: bk_create %d %s" % (path, st, lib.bk_last_error()))
    return lib, ctx, env


class _env:
    """the build's env knobs also apply while it runs (plans are built lazily)"""
    def __init__(self, env):
        self.env = env

    def __enter__(self):
        self.saved = {k: os.environ.get(k) for k in self.env}
        os.environ.update(self.env)

    def __exit__(self, *a):
        for k, v in self.saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


def kgram_ms(lib, ctx, X, n, d, ld, U, reps=3):
    lib.bk_gram_upper_device(ctx, X, _lib.BK_F64, n, d, ld, U)
    lib.bk_synchronize(ctx)
    lib.bk_timing_enable(ctx, 1)
    for _ in range(reps):
        st = lib.bk_gram_upper_device(ctx, X, _lib.BK_F64, n, d, ld, U)
        assert st == 0, lib.bk_last_error()
    lib.bk_synchronize(ctx)
    ms, cnt = ctypes.c_double(), ctypes.c_int64()
    lib.bk_timing_read(ctx, 0, ctypes.byref(ms), ctypes.byref(cnt))
    lib.bk_timing_enable(ctx, 0)
    return ms.value / max(cnt.value, 1)


def step_ms(lib, ctx, X, n, d, ld, f, sel, mean, reps=3):
    lib.bk_multikrum_device(ctx, X, _lib.BK_F64, n, d, ld, f, sel, None, mean)
    lib.bk_synchronize(ctx)
    lib.bk_timing_enable(ctx, 1)
    for _ in range(reps):
        st = lib.bk_multikrum_device(ctx, X, _lib.BK_F64, n, d, ld, f, sel, None, mean)
        assert st == 0, lib.bk_last_error()
    lib.bk_synchronize(ctx)
    out = []
    for kid in (0, 6, 3, 1, 15):  # 15: k_mean_fix (the complement path's gate)
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        if lib.bk_timing_read(ctx, kid, ctypes.byref(ms), ctypes.byref(cnt)) != 0:
            ms.value, cnt.value = 0.0, 1
        out.append(ms.value / max(cnt.value, 1))
    lib.bk_timing_enable(ctx, 0)
    # whole-step wall time with no events in the stream
    import time
    lib.bk_synchronize(ctx)
    t0 = time.perf_counter()
    for _ in range(10):
        lib.bk_multikrum_device(ctx, X, _lib.BK_F64, n, d, ld, f, sel, None, mean)
    lib.bk_synchronize(ctx)
    out.insert(4, (time.perf_counter() - t0) / 10 * 1e3)
    return out


def main_step(builds, X, n, d, f, reps):
    m = n - f
    res = {b[0]: [] for b in builds}
    outs = {}
    for label, lib, ctx, env in builds:
        outs[label] = (torch.empty(m, dtype=torch.int64, device="cuda"),
                       torch.empty(d, dtype=torch.float64, device="cuda"))
    for _ in range(reps):
        for label, lib, ctx, env in builds:
            with _env(env):
                sel, mean = outs[label]
                res[label].append(step_ms(lib, ctx, X.data_ptr(), n, d, d, f, sel.data_ptr(),
                                          mean.data_ptr()))
    torch.cuda.synchronize()
    ref = outs[builds[0][0]]
    for label, v in res.items():
        k1 = sorted(x[0] for x in v)[len(v) // 2]
        k4 = sorted(x[1] for x in v)[len(v) // 2]
        same = bool(torch.equal(outs[label][0], ref[0]) and torch.equal(outs[label][1], ref[1]))
        if not same and torch.equal(outs[label][0], ref[0]):
            scale = float(ref[1].abs().max())
            same = "sel; mean max rel %.2e" % (float((outs[label][1] - ref[1]).abs().max()) / scale)
        kfix = sorted(x[5] for x in v)[len(v) // 2]
        k2 = sorted(x[2] for x in v)[len(v) // 2]
        k1b = sorted(x[3] for x in v)[len(v) // 2]
        stp = sorted(x[4] for x in v)[len(v) // 2]
        print("%-8s n=%d d=%d f=%d step %.4f ms | K1 %.3f ms  K1b %.4f ms  K2 %.4f ms  K4 %.4f ms "
              "K4b %.4f ms  sel+mean==%s: %s" % (label, n, d, f, stp, k1, k1b, k2, k4, kfix,
                                                 builds[0][0], same),
              flush=True)


def main():
    n, d = int(os.environ.get("N", 512)), int(os.environ.get("D", 1 << 20))
    reps = int(os.environ.get("REPS", 8))
    builds = []
    for a in sys.argv[1:]:
        label, path = a.split("=", 1)
        builds.append((label,) + load(path))
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    lib0, ctx0 = builds[0][1], builds[0][2]
    lib0.bk_synth_fill_device(ctx0, X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 1, n // 3,
                              0.01, 0.05, 1e-3, 0)
    lib0.bk_synchronize(ctx0)
    if os.environ.get("F"):
        return main_step(builds, X, n, d, int(os.environ["F"]), reps)
    ue = int(lib0.bk_upper_elems(n))
    Us = {}
    for label, lib, ctx, env in builds:
        Us[label] = torch.empty(ue, dtype=torch.float64, device="cuda")
    res = {b[0]: [] for b in builds}
    for _ in range(reps):
        for label, lib, ctx, env in builds:
            with _env(env):
                res[label].append(kgram_ms(lib, ctx, X.data_ptr(), n, d, d, Us[label].data_ptr()))
    torch.cuda.synchronize()
    ref = Us[builds[0][0]]
    flops = n * (n + 1) * d
    for label, v in res.items():
        v = sorted(v)
        same = bool(torch.equal(Us[label], ref))
        print("%-8s n=%d d=%d k_gram median %.3f ms min %.3f ms (%.1f TF/s)  upper==%s: %s" %
              (label, n, d, v[len(v) // 2], v[0], flops / (v[len(v) // 2] * 1e-3) / 1e12,
               builds[0][0], same), flush=True)


if __name__ == "__main__":
    main()
