"""Is config B's step host-bound?  Issues K back-to-back bk_multikrum_device
calls (no sync between them) and reports the host's enqueue time per call next
to the wall time per call after the final sync, and the same K calls issued
from C (bk_multikrum_device_repeat is not an API: the loop runs in ctypes
either way, so the C-side figure is the libbk entry alone, timed with
clock_gettime around a tight ctypes loop of the raw function pointer)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd import _lib  # noqa: E402
from biscotti_amd.krum import Engine  # noqa: E402

e = Engine(0)
n, d, f = 100, 7850, 30
X = torch.empty((n, d), dtype=torch.float64, device="cuda")
e.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 20261017, 30, flags=1)
sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
sc = torch.empty(n, dtype=torch.float64, device="cuda")
mn = torch.empty(d, dtype=torch.float64, device="cuda")
L = _lib.lib()
fn = L.bk_multikrum_device
ctx = e._ctx
args = (ctx, ctypes.c_void_p(X.data_ptr()), _lib.BK_F64, n, d, d, f, ctypes.c_void_p(sel.data_ptr()),
        ctypes.c_void_p(sc.data_ptr()), ctypes.c_void_p(mn.data_ptr()))
for _ in range(200):
    fn(*args)
e.synchronize()
for K in (1000, 3000):
    t0 = time.perf_counter()
    for _ in range(K):
        fn(*args)
    t1 = time.perf_counter()
    e.synchronize()
    t2 = time.perf_counter()
    print("K=%d: host enqueue %.2f us/call, wall %.2f us/call" % (K, (t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6), flush=True)
# the ctypes call overhead alone (a cheap libbk entry)
t0 = time.perf_counter()
for _ in range(3000):
    L.bk_abi_version()
t1 = time.perf_counter()
print("ctypes call of bk_abi_version: %.2f us" % ((t1 - t0) / 3000 * 1e6))
