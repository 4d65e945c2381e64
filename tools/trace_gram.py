"""Per-workgroup timeline of K1 (debug): where do the cycles go?

Runs bk_gram_upper_device with BK_TRACE_FILE set (each k_gram3 workgroup
records 100 MHz start/end, shader-clock start/end, HW_ID, XCC_ID) and reports:
  * loop efficiency  = ideal MFMA cycles (nk * cost * 256) / measured cycles
  * fill efficiency  = sum of WG busy time / (CUs * makespan)
  * the distribution of per-WG durations per group.
Env: N, D, MODES (comma list of BK_GRAM_MODE values, default "0,2"); DTYPE=f32
for fp32 rows, with F32MFMA=1 on the fp32 MFMA (bk_set_f32_mode) -- its ideal
per k-block is the same cost * 256 cycles (8 MFMAs of 32 cycles per 32 columns).
"""
import collections
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from biscotti_amd import _lib  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import probe_build  # noqa: E402
probe_build.use(_lib)  # probe knobs live in the -DBK_PROBES build only
from biscotti_amd.krum import Engine  # noqa: E402

n, d = int(os.environ.get("N", 512)), int(os.environ.get("D", 1 << 20))
modes = os.environ.get("MODES", "0,2").split(",")
f32 = os.environ.get("DTYPE") == "f32"
dt = _lib.BK_F32 if f32 else _lib.BK_F64
X = torch.empty((n, d), dtype=torch.float32 if f32 else torch.float64, device="cuda")
U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
for mode in modes:
    os.environ["BK_GRAM_MODE"] = mode
    e = Engine(0)
    os.environ.pop("BK_GRAM_MODE")
    if os.environ.get("F32MFMA") == "1":
        e.set_f32_mode(_lib.BK_F32_MFMA)
    e.synth_fill_ptr(X.data_ptr(), dt, n, d, d, 0, d, 1, n // 3)
    for _ in range(3):
        e.gram_upper_ptr(X.data_ptr(), dt, n, d, d, U.data_ptr())
    e.synchronize()
    fn = tempfile.mktemp(suffix=".bin")
    os.environ["BK_TRACE_FILE"] = fn
    e.gram_upper_ptr(X.data_ptr(), dt, n, d, d, U.data_ptr())
    e.synchronize()
    os.environ.pop("BK_TRACE_FILE")
    tr = np.fromfile(fn, dtype=np.int64).reshape(-1, 24)
    os.unlink(fn)
    probe_wait, probe_bar = tr[:, 8:16], tr[:, 16:24]
    rt0, rt1, mt0, mt1, hw, xcc, gc, nk = tr[:, :8].T
    grp, gcost = gc & 0xFFFFFFFF, gc >> 32
    busy = nk > 0
    t0 = rt0.min()
    span_us = (rt1.max() - t0) / 100.0
    dur_us = (rt1 - rt0) / 100.0
    cyc = (mt1 - mt0).astype(np.float64)
    mhz = np.median(cyc[busy] / np.maximum(dur_us[busy], 1e-3))
    se = (hw >> 13) & 7
    sh = (hw >> 12) & 1
    cu = (hw >> 8) & 15
    cukey = xcc * 1000 + se * 100 + sh * 16 + cu
    ncu = len(np.unique(cukey))
    # group costs from the planner (per-SIMD MFMA units per k-step)
    costs = {int(g): int(c) for g, c in zip(grp, gcost)}
    print("mode %s: n=%d d=%d  WGs %d (busy %d) on %d CUs, makespan %.1f us, shader clock ~%.0f MHz"
          % (mode, n, d, len(tr), busy.sum(), ncu, span_us, mhz))
    fill = dur_us[busy].sum() / (ncu * span_us)
    print("  fill (sum WG time / CUs x makespan): %.3f" % fill)
    per_g = collections.defaultdict(list)
    for i in np.nonzero(busy)[0]:
        per_g[int(grp[i])].append(i)
    tot_ideal = tot_cyc = 0.0
    for g, idx in sorted(per_g.items()):
        idx = np.array(idx)
        c = costs.get(g)
        line = "  group %3d: %4d WGs  nk %5d..%5d  dur %7.1f..%7.1f us" % (
            g, len(idx), nk[idx].min(), nk[idx].max(), dur_us[idx].min(), dur_us[idx].max())
        if c:
            ideal = nk[idx] * c * 256.0
            eff = ideal / cyc[idx]
            tot_ideal += ideal.sum()
            tot_cyc += cyc[idx].sum()
            line += "  cost %d  loop eff %.3f (min %.3f)  cyc/kblock %.0f (ideal %d)" % (
                c, np.median(eff), eff.min(), np.median(cyc[idx] / nk[idx]), c * 256)
            if probe_wait[idx].any():
                pw = np.median(probe_wait[idx] / nk[idx, None], axis=0)
                pb = np.median(probe_bar[idx] / nk[idx, None], axis=0)
                line += "\n      per k-block vmcnt-wait cyc by wave %s\n      barrier cyc by wave %s" % (
                    " ".join("%5.0f" % x for x in pw), " ".join("%5.0f" % x for x in pb))
        print(line)
    if tot_cyc:
        print("  overall loop efficiency %.3f" % (tot_ideal / tot_cyc))
    # start skew: when did each CU first start / finish
    starts = (rt0[busy] - t0) / 100.0
    ends = (rt1[busy] - t0) / 100.0
    print("  WG start: first-round spread %.1f us; last WG end %.1f, first CU idle from %.1f us"
          % (np.sort(starts)[min(ncu, len(starts)) - 1], ends.max(),
             min(np.max(ends[cukey[busy] == k]) for k in np.unique(cukey[busy]))))
    # per XCD: when its CUs finish, and the clock they held (is the fill loss
    # a slow XCD, or spread within every XCD?)
    for x in np.unique(xcc[busy]):
        sel_x = busy & (xcc == x)
        cu_end = [np.max((rt1[sel_x & (cukey == k)] - t0) / 100.0) for k in np.unique(cukey[sel_x])]
        mhz_x = np.median(cyc[sel_x] / np.maximum(dur_us[sel_x], 1e-3))
        print("  XCD %d: %2d CUs  CU end %.1f..%.1f us (median %.1f)  clock %.0f MHz"
              % (x, len(cu_end), min(cu_end), max(cu_end), float(np.median(cu_end)), mhz_x))
