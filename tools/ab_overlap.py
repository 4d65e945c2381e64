"""A/B of the overlapped exchange (bk_comm_set_mode 2) at one rank's shard of
config E at N ranks, on one GPU (1-rank RCCL communicator): the serial
exchange, the overlapped one, and (probe build, BK_PIECES_NOMARK) the pieces'
workgroup order alone with no completion counts -- which part of any
difference is the order and which the counting.

    python tools/probe_build.py && python tools/ab_overlap.py [N] [reps]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    import torch
    import probe_build
    from biscotti_amd import _lib
    probe_build.use(_lib)
    import bench
    from biscotti_amd.dist import bootstrap_rccl
    from biscotti_amd.krum import Engine
    nparts = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ["BK_EMU_SPLIT_SCORES"] = str(nparts)
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    bootstrap_rccl(eng, 0, 1, lambda b, src: b)
    for rep in range(reps):
        for mode in sys.argv[3].split(",") if len(sys.argv) > 3 else ("i8x2_certified", "mfma", "exact"):
            for label, xm, knob in (("serial", 0, None), ("overlap", 2, None),
                                    ("order_only", 2, "BK_PIECES_NOMARK"),
                                    ("counts_no_wt", 2, "BK_PIECES_NOWT"),
                                    ("wait_only", 2, "BK_PIECES_NOCSTREAM"),
                                    ("counts_no_wait", 2, "BK_PIECES_NOWAIT"),
                                    ("devwait", 2, "BK_PIECES_DEVWAIT")):
                for kn in ("BK_PIECES_NOMARK", "BK_PIECES_NOWT", "BK_PIECES_NOCSTREAM",
                           "BK_PIECES_NOWAIT", "BK_PIECES_DEVWAIT"):
                    os.environ.pop(kn, None)
                if knob:
                    os.environ[knob] = "1"
                v = bench.sharded_variant(eng, dev, "E_4096x262144_fp32", mode, nparts, 0, 1,
                                          lambda: None, nparts, steps=20, warmup=5,
                                          exchange_mode=xm)
                pr = v["per_rank"][0]
                print(json.dumps({"rep": rep, "mode": mode, "exchange": label, "ms": v["ms_per_step"],
                                  "k_gram_ms": pr["k_gram_ms"], "exchange_ms": pr["exchange_ms"],
                                  "exposed_ms": pr.get("exchange_exposed_ms"),
                                  "kernels": v["kernels_ms_avg"]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
