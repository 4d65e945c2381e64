"""World-size-2 run of the dimension-sharded orchestration (biscotti_amd.dist)
on CPU with gloo: each rank builds only its column shard, computes its packed
partial Gram, the partials are all-reduced, and every rank finishes
redundantly; the result must equal the reference goldens.  On the GPU the
three hooks are libbk's bk_gram_upper_device / RCCL all-reduce /
bk_finish_device (bk_multikrum_sharded_device); here the compute hooks are the
CPU oracle and the exchange is gloo, so this checks the decomposition and the
host protocol, not the kernels (those are tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CASES = ["B_mnist", "ragged_67x1003", "honest_boundary", "n129_d4097"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, names, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here, os.path.join(here, "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cases as C
    from biscotti_amd import dist as D
    from oracle import oracle as O

    class OracleSharded(D.ShardedKrum):
        def gram_partial(self, Xl):
            return D.pack_upper(O.gram(Xl), Xl.shape[1])

        def exchange(self, U):
            t = torch.from_numpy(U.copy())
            dist.all_reduce(t)
            return t.numpy()

        def finish(self, U, Xl):
            n, f = self.n, self.f
            G = D.unpack_upper(U, n)
            dg = np.diag(G)
            Dm = (dg[:, None] + dg[None, :]) - 2.0 * G
            k = max(0, n - f - 2)
            sc = np.array([np.sum(np.sort(r)[1:1 + k]) for r in Dm])
            sel = O.select(sc, n - f)
            return sel, sc, O.mean(Xl, sel)

    out = {}
    for name in names:
        p = C.case_params(name)
        sk = OracleSharded(p["n"], p["d"], p["f"], world, rank)
        Xl = O.synth(p["n"], p["d"], p["seed"], p["nbyz"], p["mu_scale"], p["byz_scale"],
                     p["sigma"], p["flags"], c0=sk.c0, dl=sk.dl, d_total=p["d"])
        sel, sc, mean_l = sk.step(Xl)
        parts = [None] * world
        dist.all_gather_object(parts, (sk.c0, mean_l))
        out[name] = (sel, sc, np.concatenate([m for _, m in sorted(parts, key=lambda t: t[0])]))
    # the RCCL-id bootstrap rides on the same out-of-band broadcast
    from biscotti_amd.dist import torch_broadcast_bytes
    uid = torch_broadcast_bytes(bytes(range(128)) if rank == 0 else bytes(128), 0)
    out["_uid_ok"] = uid == bytes(range(128))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_matches_reference_goldens():
    import golden_util as GU
    names = [n for n in CASES if GU.have(n)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, names, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    man = GU.manifest()
    for r in (0, 1):
        assert res[r]["_uid_ok"]
        for name in names:
            g = GU.load(name)
            sel, sc, mean = res[r][name]
            assert np.array_equal(sel, g["sel"]), (r, name)
            GU.check_scores(sc, g, rel=1e-10)
            GU.check_mean(mean, g, man[name])
