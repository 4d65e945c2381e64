"""A/B of the RONI kernels (K7 logistic, K8 softmax) at bench.py's shapes, in
one process per mode: run as  python tools/roni_ab.py  (MFMA, the default) and
LIB=<another build> python tools/roni_ab.py  (an A/B build).  Prints one
JSON line with the kernel times and a hash of the score bits, so two modes can
be compared bit for bit."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from biscotti_amd import _lib
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import probe_build  # noqa: E402
    probe_build.use(_lib)  # probe knobs live in the -DBK_PROBES build only
    from biscotti_amd._lib import check, lib
    from biscotti_amd.krum import Engine
    eng = Engine(0)
    dev = torch.device("cuda:0")
    g2 = torch.Generator(device=dev).manual_seed(5)
    out = {"lib": _lib.LIB_PATH}
    nv, dr, nr = 85_000, 25, 512
    Xv = torch.randn((nv, dr), dtype=torch.float64, device=dev, generator=g2)
    yv = torch.where(torch.randn(nv, dtype=torch.float64, device=dev, generator=g2) > 0, 1.0, -1.0)
    ww = torch.randn(dr, dtype=torch.float64, device=dev, generator=g2)
    dl = torch.randn((nr, dr), dtype=torch.float64, device=dev, generator=g2) * 1e-2
    rs = torch.empty(nr, dtype=torch.float64, device=dev)
    nvm, dinm, cm, nrm = 6000, 784, 10, 100
    Xm = torch.randn((nvm, dinm), dtype=torch.float32, device=dev, generator=g2)
    ym = torch.randint(0, cm, (nvm,), dtype=torch.int32, device=dev, generator=g2)
    wm = torch.randn(cm * (dinm + 1), dtype=torch.float64, device=dev, generator=g2) * 0.05
    dm = torch.randn((nrm, cm * (dinm + 1)), dtype=torch.float64, device=dev, generator=g2) * 1e-3
    rsm = torch.empty(nrm, dtype=torch.float64, device=dev)
    ntm = torch.empty(2 * nrm + 1, dtype=torch.int32, device=dev)
    runs = {
        "k_roni": (lambda: check(lib().bk_roni_device(eng.ctx, Xv.data_ptr(), nv, dr, dr,
                                                      yv.data_ptr(), ww.data_ptr(), dl.data_ptr(),
                                                      nr, dr, rs.data_ptr())), rs,
                   2.0 * nv * (nr + 1) * dr),
        "k_roni_softmax": (lambda: check(lib().bk_roni_softmax_device(
            eng.ctx, Xm.data_ptr(), nvm, dinm, dinm, ym.data_ptr(), cm, wm.data_ptr(),
            dm.data_ptr(), nrm, cm * (dinm + 1), rsm.data_ptr(), ntm.data_ptr())), rsm,
            2.0 * nvm * (nrm + 1) * cm * dinm),
    }
    for name, (fn, res, fl) in runs.items():
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        eng.timing_enable(True)
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        t = eng.timing_read().get("k_roni")
        eng.timing_enable(False)
        ms = t["avg_ms"]
        out[name] = {"ms": round(ms, 4), "tflops": round(fl / (ms * 1e-3) / 1e12, 2),
                     "scores_sha16": hashlib.sha256(res.cpu().numpy().tobytes()).hexdigest()[:16]}
        if name == "k_roni_softmax":  # the per-evaluation near-tie counts too
            out[name]["near_sha16"] = hashlib.sha256(ntm.cpu().numpy().tobytes()).hexdigest()[:16]
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
