"""Probe of the row-fed host entry (bk_multikrum_rows) on one GPU: bench.py's
rows_entry_variant at the given configs, one JSON object per config.

    python tools/rows_probe.py [D_512x1M_f153 B_mnist A_creditcard]
    python tools/rows_probe.py --sweep B_mnist   # groups x copy kind x threads
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import bench  # noqa: E402


def main():
    import torch
    args = sys.argv[1:]
    if "--probe" in args:  # the -DBK_PROBES build (BK_ROWS_TRACE timeline)
        import probe_build
        from biscotti_amd import _lib
        probe_build.use(_lib)
    from biscotti_amd.krum import Engine
    sweep = "--sweep" in args
    names = [a for a in args if not a.startswith("--")] or ["D_512x1M_f153", "B_mnist",
                                                            "A_creditcard"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    for nm in names:
        if not sweep:
            print(json.dumps({nm: bench.rows_entry_variant(eng, dev, nm)}), flush=True)
            continue
        for kind in ("nt", "memcpy"):
            os.environ["BK_ROWS_COPY"] = kind
            for g in ("3", "4", "5", "6", "8"):
                os.environ["BK_ROWS_GROUPS"] = g
                r = bench.rows_entry_variant(eng, dev, nm, thread_sweep=(2, 4, 6, 8))
                print(json.dumps({"name": nm, "copy": kind, "groups": g,
                                  "rows_ms": r["e2e_rows_ms"], "pinned_ms": r["e2e_pinned_ms"],
                                  "serial_ms": r["e2e_rows_serial_ms"],
                                  "by_threads": r["e2e_rows_ms_by_threads"],
                                  "bitwise": r["bitwise_same_as_serial"]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
