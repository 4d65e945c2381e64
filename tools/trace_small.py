"""k_small's per-item timeline (BK_SMALL_TRACE=<file>): phase spans in us.
    BK_SMALL_TRACE=gpurun_out/small.bin python tools/trace_small.py run
    python tools/trace_small.py gpurun_out/small.bin"""
import os, sys
import numpy as np
if sys.argv[1] == "run":
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from biscotti_amd import _lib
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import probe_build  # noqa: E402
    probe_build.use(_lib)  # probe knobs live in the -DBK_PROBES build only
    from biscotti_amd.krum import Engine
    tf = os.environ["BK_SMALL_TRACE"]
    if os.path.exists(tf):
        os.remove(tf)
    e = Engine(0)
    n, d, f = 100, 7850, 30
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    e.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, 20261017, 30, flags=1)
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mn = torch.empty(d, dtype=torch.float64, device="cuda")
    os.environ.pop("BK_SMALL_TRACE")
    for _ in range(200):  # warm the clock without tracing, then trace one call
        e.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(), sc.data_ptr(), mn.data_ptr())
    os.environ["BK_SMALL_TRACE"] = tf
    for _ in range(1):
        e.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(), sc.data_ptr(), mn.data_ptr())
    e.synchronize()
    sys.argv[1] = tf
raw = np.fromfile(sys.argv[1], dtype=np.int64)
pos, calls = 0, []
while pos < len(raw):
    items, P, Q, nS, C, grid = raw[pos:pos + 6]
    tr = raw[pos + 6:pos + 6 + 8 * items].reshape(items, 8)
    wg = raw[pos + 6 + 8 * items:pos + 6 + 8 * items + 2 * grid].reshape(grid, 2)
    calls.append((P, Q, nS, C, tr, wg))
    pos += 6 + 8 * items + 2 * grid
P, Q, nS, C, tr, wg = calls[-1]
t0 = tr[:, 0][tr[:, 0] > 0].min()
us = lambda x: (x - t0) / 100.0  # s_memrealtime: 100 MHz
kinds = [("G", 0, P), ("R", P, P + Q), ("S", P + Q, P + Q + nS), ("M", P + Q + nS, P + Q + nS + C)]
for name, a, b in kinds:
    seg = tr[a:b]
    if len(seg) == 0:
        continue
    st, wt, en = us(seg[:, 0]), us(seg[:, 1]), us(seg[:, 2])
    work = en - np.where(seg[:, 1] > 0, wt, st)
    print("%s items %3d: start %6.2f..%6.2f  waited-until %6.2f..%6.2f  end %6.2f..%6.2f  work med %.2f max %.2f us"
          % (name, b - a, st.min(), st.max(), (wt.min() if name != "G" else 0), (wt.max() if name != "G" else 0), en.min(), en.max(), np.median(work), work.max()))
    if (seg[:, 6] > 0).all() and (seg[:, 7] > 0).all():
        s0, s1 = us(seg[:, 6]), us(seg[:, 7])
        b0 = np.where(seg[:, 1] > 0, wt, st)
        print("    in-item stages (median us): to stamp 0 %.2f, stamp 0->1 %.2f, stamp 1->end %.2f"
              % (np.median(s0 - b0), np.median(s1 - s0), np.median(en - s1)))
clk = (tr[:, 5] - tr[:, 4]) / np.maximum(1, tr[:, 2] - tr[:, 0]) * 100 / 1000.0
print("shader clock (GHz) over items: median %.2f min %.2f" % (np.median(clk[clk > 0]), clk[clk > 0].min()))
print("calls traced: %d; last call span %.2f us" % (len(calls), us(tr[:, 2]).max()))
print("workgroups %d: entry %.2f..%.2f us (first item at 0), exit %.2f..%.2f us"
      % (len(wg), us(wg[:, 0]).min(), us(wg[:, 0]).max(), us(wg[:, 1]).min(), us(wg[:, 1]).max()))
