"""Two processes on the one MI355X drive libbk's SHARDED entries:
each rank generates only its column shard on the device, computes its packed
partial Gram with bk_gram_upper_device, the partials are summed across the two
processes with gloo (RCCL cannot put two ranks on one device; on an 8-GPU node
the same exchange is libbk's ncclAllReduce), and each rank finishes with
bk_finish_device -- scores and selection redundantly, the mean of its own
columns.  The selection must equal the reference golden bit-exactly, on every
rank, and the concatenated means must be within the §8(d) bound.  This is the
product path of SURVEY.md §8(e) across processes, which
tests/test_dist_gloo.py (oracle hooks) does not exercise."""
import os
import socket

import numpy as np
import pytest

import golden_util as GU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = [c for c in ("C_1024x131072", "D_512x1M_f256", "C_tight", "B_mnist") if GU.have(c)]


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
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cases as C
        from biscotti_amd import _lib
        from biscotti_amd.dist import shard_bounds
        from biscotti_amd.krum import Engine
        eng = Engine(0)
        out = {}
        for name in names:
            p = C.case_params(name)
            n, d, f = p["n"], p["d"], p["f"]
            c0, dl = shard_bounds(d, world, rank)
            X = torch.empty((n, max(dl, 1)), dtype=torch.float64, device="cuda")
            eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, dl, X.stride(0), c0, d, p["seed"],
                               p["nbyz"], p["mu_scale"], p["byz_scale"], p["sigma"], p["flags"])
            usz = int(_lib.lib().bk_upper_elems(n))
            U = torch.empty(usz, dtype=torch.float64, device="cuda")
            eng.gram_upper_ptr(X.data_ptr(), _lib.BK_F64, n, dl, X.stride(0), U.data_ptr())
            eng.synchronize()
            Uh = U.cpu()
            dist.all_reduce(Uh)  # the exchange (RCCL all-reduce on a multi-GPU node)
            U.copy_(Uh)
            sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
            sc = torch.empty(n, dtype=torch.float64, device="cuda")
            mean = torch.empty(max(dl, 1), dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            eng.finish_ptr(U.data_ptr(), X.data_ptr(), _lib.BK_F64, n, dl, X.stride(0), f,
                           sel.data_ptr(), sc.data_ptr(), mean.data_ptr())
            eng.synchronize()
            mg = eng.selection_margin()
            parts = [None] * world
            dist.all_gather_object(parts, (c0, mean[:dl].cpu().numpy()))
            full_mean = np.concatenate([m for _, m in sorted(parts, key=lambda t: t[0])])
            out[name] = (sel.cpu().numpy(), sc.cpu().numpy(), full_mean, mg, float(Uh[-4]))
            del X, U
            torch.cuda.empty_cache()
        eng.close()
        q.put((rank, out))
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.skipif(not CASES, reason="goldens not generated")
def test_two_process_sharded_product_path():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, CASES, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    man = GU.manifest()
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
        for name in CASES:
            g = GU.load(name)
            sel, sc, mean, mg, dsum = res[r][name]
            p = GU.C.case_params(name)
            assert dsum == p["d"]  # the trailing pairs summed to the total d
            assert np.array_equal(sel, g["sel"]), (r, name)
            GU.check_scores(sc, g, rel=1e-9)
            GU.check_mean(mean, g, man[name])
            GU.check_margin(mg, sc, g["sq"], p["n"], p["f"], p["d"])
            assert not mg["near_tie"]
    # both ranks selected identically (the redundant finish)
    for name in CASES:
        assert np.array_equal(res[0][name][0], res[1][name][0])
        assert np.array_equal(res[0][name][1], res[1][name][1])


def _poison_worker(rank, world, port, q):
    """Rank 1's partial Gram fails (test knob BK_TEST_FAIL_BEFORE_EXCHANGE=2):
    its bk_gram_upper_device returns the error and poisons the partial, the
    rank still joins the exchange (so rank 0 is not left waiting), and both
    ranks' finishes report the call invalid (BK_ERCCL) instead of selecting
    from a wrong Gram."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here, os.path.join(here, "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    if rank == 1:
        os.environ["BK_TEST_FAIL_BEFORE_EXCHANGE"] = "2"
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from biscotti_amd import _lib
        from biscotti_amd.dist import shard_bounds
        from biscotti_amd.krum import Engine
        eng = Engine(0)
        n, d, f = 300, 20000, 90
        c0, dl = shard_bounds(d, world, rank)
        X = torch.empty((n, dl), dtype=torch.float64, device="cuda")
        eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, dl, dl, c0, d, 99, 60)
        U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
        gram_status = 0
        try:
            eng.gram_upper_ptr(X.data_ptr(), _lib.BK_F64, n, dl, dl, U.data_ptr())
        except _lib.BKError as e:
            gram_status = e.status
        torch.cuda.synchronize()
        Uh = U.cpu()
        dist.all_reduce(Uh)  # joined by both ranks, whatever happened before
        U.copy_(Uh)
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        eng.finish_ptr(U.data_ptr(), X.data_ptr(), _lib.BK_F64, n, dl, dl, f, sel.data_ptr())
        fin_status = 0
        try:
            eng.synchronize()
        except _lib.BKError as e:
            fin_status = e.status
        eng.close()
        q.put((rank, (gram_status, fin_status)))
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_two_process_failed_rank_poisons_instead_of_stranding():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_poison_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == (0, -4), res  # rank 0: its Gram fine, the summed record invalid
    assert res[1] == (-3, -4), res  # rank 1: its own error, then the same verdict
