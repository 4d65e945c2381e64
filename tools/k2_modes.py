"""Timing-only split of K2 (BK_K2_MODE: 0 full, 1 loads+keys only, 2 sort of
synthetic keys only) at E's shard shape and D's: one process per mode."""
import ctypes, os, subprocess, sys
if len(sys.argv) > 1:
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from biscotti_amd import _lib
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import probe_build
    probe_build.use(_lib)  # probe knobs live in the -DBK_PROBES build only
    from biscotti_amd.krum import Engine
    eng = Engine(0)
    for (n, d, f, dt, tdt) in [(4096, 8192, 1228, _lib.BK_F32, torch.float32), (512, 65536, 153, _lib.BK_F64, torch.float64), (100, 7850, 30, _lib.BK_F64, torch.float64)]:
        X = torch.empty((n, d), dtype=tdt, device="cuda")
        eng.synth_fill_ptr(X.data_ptr(), dt, n, d, d, 0, d, 5, f)
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        for rep in range(2):
            eng.timing_enable(bool(rep))
            for _ in range(10 if rep else 2):
                eng.multikrum_device_ptr(X.data_ptr(), dt, n, d, d, f, sel.data_ptr())
            eng.synchronize()
        t = eng.timing_read()
        if "k_scores" in t:  # (n <= 128 runs k_small, no K2)
            print("mode %s n=%d k_scores %.4f ms" % (os.environ.get("BK_K2_MODE", "0"), n, t["k_scores"]["avg_ms"]), flush=True)
else:
    for m in ("0", "1", "2"):
        subprocess.run([sys.executable, __file__, "x"], env=dict(os.environ, BK_K2_MODE=m), check=True)
