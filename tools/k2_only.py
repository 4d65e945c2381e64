"""Config E's 8-rank shard shape (n = 4096, d = 8192 fp32) through
bk_multikrum_device a few times: a short target for K2 (k_scores) PMC passes.
    rocprofv3 --pmc <counters> --kernel-trace -- python3 tools/k2_only.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd import _lib  # noqa: E402
from biscotti_amd.krum import Engine  # noqa: E402

e = Engine(0)
n, d, f = 4096, 8192, 1228
X = torch.empty((n, d), dtype=torch.float32, device="cuda")
e.synth_fill_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, 0, d, 5, f)
sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
for _ in range(int(os.environ.get("K2_REPS", "4"))):
    e.multikrum_device_ptr(X.data_ptr(), _lib.BK_F32, n, d, d, f, sel.data_ptr())
e.synchronize()
print("done")
