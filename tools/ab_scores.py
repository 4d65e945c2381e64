"""A/B of K2 (k_scores) between two libbk.so builds in one process: the scores
must be bitwise equal (any correct sort yields the same sorted keys) and the
K2 time is compared on D's and E's 8-GPU shard shapes.
    python tools/ab_scores.py build_ab/libbk_base.so biscotti_amd/libbk.so"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd import _lib  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    ctx = ctypes.c_void_p()
    assert lib.bk_create(ctypes.byref(ctx), 0) == 0
    if hasattr(lib, "bk_set_small_path"):  # K2 is the subject: n <= 128 through the chain too
        assert lib.bk_set_small_path(ctx, 0) == 0
    return lib, ctx


libs = [load(p) for p in sys.argv[1:3]]
dev = torch.device("cuda", 0)
for (n, d, f, dt, tdt, seed) in [(512, 131072, 153, _lib.BK_F64, torch.float64, 20261019),
                                 (4096, 32768, 1228, _lib.BK_F32, torch.float32, 20261020),
                                 (1024, 16384, 307, _lib.BK_F64, torch.float64, 3),
                                 (100, 7850, 30, _lib.BK_F64, torch.float64, 4),
                                 (3000, 4096, 900, _lib.BK_F64, torch.float64, 5)]:
    X = torch.empty((n, d), dtype=tdt, device=dev)
    L0, c0 = libs[0]
    assert L0.bk_synth_fill_device(c0, ctypes.c_void_p(X.data_ptr()), dt, n, d, d, 0, d, seed,
                                   f, 0.01, 0.05, 1e-3, 0) == 0
    L0.bk_synchronize(c0)
    out = []
    for L, c in libs:
        sel = torch.empty(n - f, dtype=torch.int64, device=dev)
        sc = torch.empty(n, dtype=torch.float64, device=dev)
        for rep in range(2):
            L.bk_timing_enable(c, 1 if rep else 0)
            for _ in range(10 if rep else 2):
                assert L.bk_multikrum_device(c, ctypes.c_void_p(X.data_ptr()), dt, n, d, d, f,
                                             ctypes.c_void_p(sel.data_ptr()),
                                             ctypes.c_void_p(sc.data_ptr()), None) == 0
            L.bk_synchronize(c)
        tot = 0.0
        for kname in ("k_scores", "k_transpose"):  # k_transpose: id 2 (v2, large n)
            ms, cnt = ctypes.c_double(), ctypes.c_int64()
            L.bk_timing_read(c, _lib.K[kname], ctypes.byref(ms), ctypes.byref(cnt))
            tot += ms.value / max(cnt.value, 1) if cnt.value else 0.0
        out.append((sel.cpu().numpy(), sc.cpu().numpy(), tot))
    same = np.array_equal(out[0][1].view(np.int64), out[1][1].view(np.int64)) and \
        np.array_equal(out[0][0], out[1][0])
    print("n=%5d d=%6d: k_scores(+k_transpose) base %.4f ms  new %.4f ms  scores+selection bitwise %s"
          % (n, d, out[0][2], out[1][2], same), flush=True)
    assert same
