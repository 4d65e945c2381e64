"""K4 (the masked mean) at config D, timed with libbk's events over back-to-back
Multi-Krum steps: an A/B of k_mean build variants (e.g. BK_MEAN_DEPTH).

    LIB=tools/ab/libbk_d16.so python tools/k4_probe.py [steps]   (default: the product libbk.so)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    import torch
    import bench
    from biscotti_amd import _lib
    if os.environ.get("LIB"):
        import probe_build
        probe_build.use(_lib)
    from biscotti_amd.krum import Engine
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    w = bench.WORKLOADS["D_512x1M_f153"]
    n, d, f = w["n"], w["d"], w["f"]
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, w["seed"], w["nbyz"])
    sel = torch.empty(n - f, dtype=torch.int64, device=dev)
    mean = torch.empty(d, dtype=torch.float64, device=dev)
    out = []
    for rep in range(3):
        for _ in range(10):
            eng.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(), 0,
                                     mean.data_ptr())
        torch.cuda.synchronize()
        eng.timing_select(["k_mean"])
        for _ in range(steps):
            eng.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(), 0,
                                     mean.data_ptr())
        torch.cuda.synchronize()
        out.append(eng.timing_read()["k_mean"]["avg_ms"])
        eng.timing_select([])
    h = __import__("hashlib").sha256(mean.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "k_mean_ms": out, "mean_sha16": h}),
          flush=True)
    eng.close()


if __name__ == "__main__":
    main()
