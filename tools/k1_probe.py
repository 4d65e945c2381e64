"""K1 at one planner / build configuration, measured the way clock-sensitive
changes must be (MI355X_MICROARCH.md 'DVFS give-back'): in a process of its
own, after >= WARM seconds of back-to-back launches, then TIMED launches on
HIP events, then one traced launch for the in-kernel clock (s_memtime over
s_memrealtime per workgroup, per XCD).  Interleaving builds in one process
(tools/ab_libs.py) blends their power states: r3's L2-window ablation read
-0.3% there and -6% (clock 2.20 -> 2.35 GHz) in separate processes.

    env [BK_PLAN_MODE=..] [BK_PLAN_ROUNDS=..] [LIB=build.so] N=512 D=1048576 \
        python tools/k1_probe.py <label>

Prints one JSON line: label, K1 median/min ms, TF/s, frac of 78.6, median
clock over workgroups, HBM bytes are NOT measured here (PMC: tools/profile.sh).
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd import _lib  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import probe_build  # noqa: E402
probe_build.use(_lib)  # probe knobs live in the -DBK_PROBES build only
from biscotti_amd.krum import Engine  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else "k1"
n, d = int(os.environ.get("N", 512)), int(os.environ.get("D", 1 << 20))
warm_s = float(os.environ.get("WARM", 2.0))
timed = int(os.environ.get("TIMED", 20))
f32 = os.environ.get("DTYPE") == "f32"
dt = _lib.BK_F32 if f32 else _lib.BK_F64
X = torch.empty((n, d), dtype=torch.float32 if f32 else torch.float64, device="cuda")
U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
e = Engine(0)
if os.environ.get("F32MFMA") == "1":
    e.set_f32_mode(_lib.BK_F32_MFMA)
e.synth_fill_ptr(X.data_ptr(), dt, n, d, d, 0, d, 1, n // 3)


def run(k):
    for _ in range(k):
        e.gram_upper_ptr(X.data_ptr(), dt, n, d, d, U.data_ptr())


run(2)
e.synchronize()
t0 = time.perf_counter()
while time.perf_counter() - t0 < warm_s:
    run(5)
    e.synchronize()
e.timing_select(["k_gram"])
run(timed)
e.synchronize()
tr = e.timing_read()["k_gram"]
e.timing_select([])
# per-call times: re-run with events on each (the same as the bench's K1 events)
per = []
for _ in range(timed):
    e.timing_select(["k_gram"])
    run(1)
    e.synchronize()
    per.append(e.timing_read()["k_gram"]["avg_ms"])
e.timing_select([])
# one traced launch right after: the in-kernel clock per workgroup
fd, path = tempfile.mkstemp(prefix="k1trace_")
os.close(fd)
os.environ["BK_TRACE_FILE"] = path
run(1)
e.synchronize()
os.environ.pop("BK_TRACE_FILE")
raw = np.fromfile(path, dtype=np.int64)
os.unlink(path)
rec = raw.reshape(-1, 24)
rt = (rec[:, 1] - rec[:, 0]).astype(np.float64)
mt = (rec[:, 3] - rec[:, 2]).astype(np.float64)
ok = rt > 0
clk = mt[ok] / rt[ok] * 0.1  # GHz (s_memrealtime runs at 100 MHz)
flops = n * (n + 1) * d
med = float(np.median(per))
print(json.dumps({"label": label, "n": n, "d": d, "env": {k: v for k, v in os.environ.items()
                                                          if k.startswith("BK_") or k == "LIB"},
                  "k1_avg_ms": round(tr["avg_ms"], 4), "k1_median_ms": round(med, 4),
                  "k1_min_ms": round(float(np.min(per)), 4),
                  "tflops": round(flops / (med * 1e-3) / 1e12, 2),
                  "frac_of_78.6": round(flops / (med * 1e-3) / 1e12 / 78.6, 4),
                  "clock_ghz_median": round(float(np.median(clk)), 3),
                  "clock_ghz_p10_p90": [round(float(np.percentile(clk, 10)), 3),
                                        round(float(np.percentile(clk, 90)), 3)]}), flush=True)
e.close()
