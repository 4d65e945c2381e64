"""Probe: does a column sum over all n rows, run on a
second stream concurrently with K1, slow K1 down?  If not, K4 could read only
the f rejected rows (mean = (sum_all - sum_rejected) / m).  Config D."""
import time

import numpy as np
import torch

from biscotti_amd import _lib
from biscotti_amd.krum import Engine

n, d, f = 512, 1 << 20, 153
m = n - f
dev = torch.device("cuda", 0)
eng = Engine(0)   # its own stream
side = Engine(0)  # a second context = a second stream
X = torch.empty((n, d), dtype=torch.float64, device=dev)
eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 20261015 + 4, 153)
eng.synchronize()
sel = torch.empty(m, dtype=torch.int64, device=dev)
mean = torch.empty(d, dtype=torch.float64, device=dev)
allidx = torch.arange(n, dtype=torch.int64, device=dev)
colsum = torch.zeros(d, dtype=torch.float64, device=dev)
torch.cuda.synchronize()


def krum():
    eng.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(), None,
                             mean.data_ptr())


def cs():
    side.aggregate_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, allidx.data_ptr(), n,
                              colsum.data_ptr())


for _ in range(5):
    krum()
    cs()
eng.synchronize()
side.synchronize()
for label, conc in (("alone", False), ("with concurrent colsum", True), ("alone", False),
                    ("with concurrent colsum", True)):
    eng.timing_enable(True)
    side.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(20):
        if conc:
            cs()
        krum()
    eng.synchronize()
    side.synchronize()
    t = (time.perf_counter() - t0) / 20 * 1e3
    kt = eng.timing_read()
    st = side.timing_read()
    print("%-24s step %.3f ms  k_gram %.3f ms  k_mean %.3f ms  colsum %s" % (
        label, t, kt["k_gram"]["avg_ms"], kt["k_mean"]["avg_ms"],
        "%.3f ms" % st["k_aggregate"]["avg_ms"] if "k_aggregate" in st else "-"), flush=True)
side.timing_enable(True)
for _ in range(20):
    cs()
side.synchronize()
print("colsum alone %.3f ms" % side.timing_read()["k_aggregate"]["avg_ms"], flush=True)
