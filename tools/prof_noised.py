"""Profile target for bk_multikrum_noised at config D (512 x 2^20 fp64, k = 1):
run under `rocprofv3 --kernel-trace --memory-copy-trace --stats` to see the
chunked H2D copies overlap K6 ("Noise fused into the staging")."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from biscotti_amd import _lib  # noqa: E402
from biscotti_amd.krum import Engine  # noqa: E402

n, d, k, f = 512, 1 << 20, 1, 153
dev = torch.device("cuda", 0)
eng = Engine(0)
X = torch.empty((n, d), dtype=torch.float64, device=dev)
eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 20261015 + 4, 153)
Dh = torch.empty((n, d), dtype=torch.float64, pin_memory=True)
Dh.copy_(X)
Nh = torch.empty((n, k, d), dtype=torch.float64, pin_memory=True)
Nh.copy_(torch.randn((n, k, d), dtype=torch.float64, device=dev) * 1e-4)
del X
torch.cuda.synchronize()
sel = np.empty(n - f, dtype=np.int64)
mean = np.empty(d, dtype=np.float64)
for it in range(4):
    t0 = time.perf_counter()
    eng.multikrum_noised_ptr(Dh.data_ptr(), d, Nh.data_ptr(), k, d, _lib.BK_HOST_PINNED, n, d, f,
                             sel.ctypes.data, None, mean.ctypes.data)
    print("call %d: %.2f ms" % (it, (time.perf_counter() - t0) * 1e3), flush=True)

# K1 on the same noised batch, device-resident: back to back, and after an idle
# gap as long as the staging (is the slower K1 after the copies a clock ramp?)
Xn = torch.empty((n, d), dtype=torch.float64, device=dev)
Nd = Nh.cuda()
Dg = Dh.cuda()
torch.cuda.synchronize()  # the engine runs on its own stream
eng.noise_apply_ptr(Dg.data_ptr(), n, d, d, Nd.data_ptr(), k, d, Xn.data_ptr(), d)
eng.synchronize()
del Nd, Dg
dsel = torch.empty(n - f, dtype=torch.int64, device=dev)
dmean = torch.empty(d, dtype=torch.float64, device=dev)


def dev_step():
    eng.multikrum_device_ptr(Xn.data_ptr(), _lib.BK_F64, n, d, d, f, dsel.data_ptr(), None,
                             dmean.data_ptr())


eng.timing_enable(True)
for _ in range(4):
    dev_step()
eng.synchronize()
print("back to back: k_gram avg %.3f ms" % eng.timing_read()["k_gram"]["avg_ms"], flush=True)
eng.timing_enable(True)
for _ in range(4):
    time.sleep(0.15)
    dev_step()
    eng.synchronize()
print("after 150 ms idle: k_gram avg %.3f ms" % eng.timing_read()["k_gram"]["avg_ms"], flush=True)
eng.timing_enable(True)
for _ in range(4):
    Dh2 = Dh.cuda(non_blocking=True)  # a 4.3 GB H2D copy right before, like the staging
    torch.cuda.synchronize()
    dev_step()
    eng.synchronize()
    del Dh2
print("after a 4.3 GB H2D copy: k_gram avg %.3f ms" % eng.timing_read()["k_gram"]["avg_ms"],
      flush=True)
same = np.array_equal(dsel.cpu().numpy(), sel)
print("device path selection == noised path selection:", same, flush=True)
eng.close()
