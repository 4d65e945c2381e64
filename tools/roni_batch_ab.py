"""k_roni_batch (bk_roni_softmax_batches_device, the torch-path RONI with the
reference's last-mini-batch semantics) at bench.py's shape for one build of
libbk.so, in a process of its own:

    LIB=<build> python tools/roni_batch_ab.py <label>

Prints one JSON line: the median time of 20 calls and a hash of the scores and
near-tie counts, so two builds can be compared bit for bit."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd import _lib  # noqa: E402

if os.environ.get("LIB"):
    _lib.LIB_PATH = os.path.abspath(os.environ["LIB"])


def main():
    import torch
    from biscotti_amd._lib import check, lib
    from biscotti_amd.krum import Engine
    torch.zeros(1, device="cuda")
    eng = Engine(0)
    dev = torch.device("cuda:0")
    g2 = torch.Generator(device=dev).manual_seed(5)
    nvm, dinm, cm, nrm, nbm = 6000, 784, 10, 100, int(os.environ.get("NB", 10))
    Xm = torch.randn((nvm, dinm), dtype=torch.float32, device=dev, generator=g2)
    ym = torch.randint(0, cm, (nvm,), dtype=torch.int32, device=dev, generator=g2)
    wm = torch.randn(cm * (dinm + 1), dtype=torch.float64, device=dev, generator=g2) * 0.05
    dm = torch.randn((nrm, cm * (dinm + 1)), dtype=torch.float64, device=dev, generator=g2) * 1e-3
    im = torch.randint(0, nvm, (nrm, 2, nbm), dtype=torch.int64, device=dev, generator=g2)
    rs = torch.empty(nrm, dtype=torch.float64, device=dev)
    nt = torch.empty(2 * nrm + 1, dtype=torch.int32, device=dev)

    def run():
        check(lib().bk_roni_softmax_batches_device(
            eng.ctx, Xm.data_ptr(), nvm, dinm, dinm, ym.data_ptr(), cm, wm.data_ptr(),
            dm.data_ptr(), nrm, cm * (dinm + 1), im.data_ptr(), nbm, rs.data_ptr(), nt.data_ptr()))
    for _ in range(5):
        run()
    eng.synchronize()
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        run()
        eng.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    h = hashlib.sha256(rs.cpu().numpy().tobytes() + nt.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"label": sys.argv[1] if len(sys.argv) > 1 else "x", "nb": nbm,
                      "ms_median": round(sorted(ts)[len(ts) // 2], 4), "hash": h}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
