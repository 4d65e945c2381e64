"""A/B builds of libbk.so on K6 (noise application) at the bench's shape:
128 updates x 2^20 fp64, k = 2 noise vectors (bench.py next_rows).
    python tools/ab_noise.py a=lib1.so b=lib2.so"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ab_libs import load  # noqa: E402

rows, k, d = 128, 2, 1 << 20
delta = torch.randn((rows, d), dtype=torch.float64, device="cuda")
noise = torch.randn((rows * k, d), dtype=torch.float64, device="cuda")
out = torch.empty((rows, d), dtype=torch.float64, device="cuda")
builds = [(a.split("=", 1)[0],) + load(a.split("=", 1)[1]) for a in sys.argv[1:]]
res = {b[0]: [] for b in builds}
ref = None
for rep in range(8):
    for label, lib, ctx, env in builds:
        lib.bk_timing_enable(ctx, 1)
        for _ in range(5):
            assert lib.bk_noise_apply_device(ctx, delta.data_ptr(), rows, d, d, noise.data_ptr(), k, d,
                                             out.data_ptr(), d) == 0
        lib.bk_synchronize(ctx)
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        lib.bk_timing_read(ctx, 13, ctypes.byref(ms), ctypes.byref(cnt))
        lib.bk_timing_enable(ctx, 0)
        res[label].append(ms.value / cnt.value)
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref)
for label, v in res.items():
    v = sorted(v)
    ms = v[len(v) // 2]
    print("%-8s k_noise median %.4f ms  %.1f GB/s" % (label, ms, rows * d * 8 * (k + 2) / ms / 1e6))
