"""Timing-only ablations of K1 (wrong results by design): normal / no-MFMA /
no-global-load builds of k_gram3, interleaved in one process (rule 24)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd import _lib  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_build  # noqa: E402
probe_build.use(_lib)  # probe knobs live in the -DBK_PROBES build only
from biscotti_amd.krum import Engine  # noqa: E402

n, d = int(os.environ.get("N", 512)), int(os.environ.get("D", 1 << 20))
engines = {}
for mode in ("0", "1", "2"):
    os.environ["BK_GRAM_MODE"] = mode
    engines[mode] = Engine(0)
os.environ.pop("BK_GRAM_MODE")
pad = int(os.environ.get("LDPAD", 0))
ld = d + pad
X = torch.empty((n, ld), dtype=torch.float64, device="cuda")
e0 = engines["0"]
e0.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, ld, 0, d, 1, n // 3)
U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
res = {m: [] for m in engines}
for rnd in range(6):
    for m, e in engines.items():
        e.gram_upper_ptr(X.data_ptr(), _lib.BK_F64, n, d, ld, U.data_ptr())
        e.synchronize()
        e.timing_enable(True)
        for _ in range(3):
            e.gram_upper_ptr(X.data_ptr(), _lib.BK_F64, n, d, ld, U.data_ptr())
        t = e.timing_read()
        e.timing_enable(False)
        res[m].append(t["k_gram"]["avg_ms"])
flops = n * (n + 1) * d
for m, v in res.items():
    v = sorted(v)
    print("ld=%d mode %s: median %.3f ms  min %.3f ms  (%.1f TF/s at median)" %
          (ld, m, v[len(v) // 2], v[0], flops / (v[len(v) // 2] * 1e-3) / 1e12), flush=True)
