"""What a single host-entry call at config B pays after the GPU has idled,
piece by piece: each measurement follows IDLE seconds of idle, REPS times,
medians printed as one JSON line.

  h2d        the 6.28 MB pinned -> device copy alone (torch copy_, synchronize)
  device     bk_multikrum_device on the resident batch (k_small), synchronize
  host       bk_multikrum(BK_HOST_PINNED): copy + kernel + outputs
  wake+host  a 1-element torch kernel, synchronize, then the host entry
             (does waking the GPU first help, and what does the wake cost?)
  prewarm1ms_host  a tiny asynchronous Multi-Krum launch, 1 ms of sleep, then
             the host entry (timed): a verifier waking the GPU as the first
             update of a batch arrives
  warm_host  the host entry back to back (no idle), for scale

    python tools/idle_probe.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd import _lib  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_build  # noqa: E402
probe_build.use(_lib)  # probe knobs live in the -DBK_PROBES build only
from biscotti_amd.krum import Engine  # noqa: E402

IDLE = float(os.environ.get("IDLE", 0.2))
REPS = int(os.environ.get("REPS", 9))
n, d, f = 100, 7850, 30
m = n - f
torch.zeros(1, device="cuda")
eng = Engine(0)
Xd = torch.empty((n, d), dtype=torch.float64, device="cuda")
eng.synth_fill_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 20261017, 30, flags=1)
Xh = torch.empty((n, d), dtype=torch.float64, pin_memory=True)
Xh.copy_(Xd)
seld = torch.empty(m, dtype=torch.int64, device="cuda")
meand = torch.empty(d, dtype=torch.float64, device="cuda")
selh = np.empty(m, dtype=np.int64)
meanh = np.empty(d, dtype=np.float64)
mo = ctypes.c_int64(0)
L = _lib.lib()
tiny = torch.zeros(1, device="cuda")


def host():
    _lib.check(L.bk_multikrum(eng.ctx, ctypes.c_void_p(Xh.data_ptr()), _lib.BK_HOST_PINNED,
                              _lib.BK_F64, n, d, d, f, selh.ctypes.data, ctypes.addressof(mo),
                              None, meanh.ctypes.data))


def device():
    eng.multikrum_device_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, f, seld.data_ptr(), None,
                             meand.data_ptr())
    eng.synchronize()


def h2d():
    Xd.copy_(Xh, non_blocking=True)
    torch.cuda.synchronize()


def wake_host():
    tiny.add_(1.0)
    torch.cuda.synchronize()
    host()


Xt = torch.zeros((4, 8), dtype=torch.float64, device="cuda")
selt = torch.empty(2, dtype=torch.int64, device="cuda")


def prewarm_host():
    # what a verifier could do when its first update arrives: one tiny
    # asynchronous launch on the engine's stream, then the batch 1 ms later
    # (the prewarm is outside the timed call, as it would be in the verifier)
    eng.multikrum_device_ptr(Xt.data_ptr(), _lib.BK_F64, 4, 8, 8, 2, selt.data_ptr())
    time.sleep(0.001)


for _ in range(50):
    host()
    device()
res = {}
for name, fn, pre in (("h2d", h2d, None), ("device", device, None), ("host", host, None),
                      ("wake+host", wake_host, None), ("prewarm1ms_host", host, prewarm_host)):
    ts = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        time.sleep(IDLE)
        if pre:
            pre()
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    res[name + "_us"] = round(float(np.median(ts)), 1)
    res[name + "_all_us"] = [round(x, 1) for x in ts]
ts = []
for _ in range(200):
    t0 = time.perf_counter()
    host()
    ts.append((time.perf_counter() - t0) * 1e6)
res["warm_host_us"] = round(float(np.median(ts)), 1)
print(json.dumps({"idle_s": IDLE, **res}), flush=True)
eng.close()
