"""libbk's multi-rank RCCL path with real ranks, one GPU each:
bk_multikrum_sharded_device at n > 2048, where every rank scores only its
share of the rows and one in-place ncclAllGather of {scores, status} hands
every rank all n scores (split scoring).

Needs >= 2 visible GPUs: skipped on the 1-GPU box (where the same arithmetic
is covered by tests/test_gpu_parity.py::test_split_scores_* through a 1-rank
communicator scoring in R shares).  Checks, on each of 2 ranks:
  * selection and scores bitwise those of the unsplit finish (bk_finish_device
    on one GPU) over the same summed Gram (the two shards' partials, U0 + U1 --
    the all-reduce's sum at two ranks), and the shard means within §8(d);
  * a rank whose share fails (BK_TEST_SPLIT_FAIL) still joins the all-gather,
    and every rank reports the call invalid (BK_ERCCL; the failing rank its
    own error) instead of selecting from stale scores."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

N, D, F = 2500, 4096, 750


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fail_rank, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    if fail_rank is not None:
        os.environ["BK_TEST_SPLIT_FAIL"] = str(fail_rank + 1)
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from biscotti_amd import _lib
        from biscotti_amd.dist import bootstrap_rccl, shard_bounds, torch_broadcast_bytes
        from biscotti_amd.krum import Engine
        eng = Engine(rank)
        bootstrap_rccl(eng, rank, world, torch_broadcast_bytes)
        c0, dl = shard_bounds(D, world, rank)
        X = torch.empty((N, dl), dtype=torch.float64, device="cuda")
        eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, N, dl, dl, c0, D, 2500, F)
        sel = torch.empty(N - F, dtype=torch.int64, device="cuda")
        sc = torch.empty(N, dtype=torch.float64, device="cuda")
        mean = torch.empty(dl, dtype=torch.float64, device="cuda")
        status = 0
        try:
            eng.multikrum_sharded_ptr(X.data_ptr(), _lib.BK_F64, N, dl, dl, F, sel.data_ptr(),
                                      sc.data_ptr(), mean.data_ptr())
            eng.synchronize()
        except _lib.BKError as e:
            status = e.status
        # this rank's partial Gram, for the parent's unsplit reference
        U = torch.empty(int(_lib.lib().bk_upper_elems(N)), dtype=torch.float64, device="cuda")
        eng.gram_upper_ptr(X.data_ptr(), _lib.BK_F64, N, dl, dl, U.data_ptr())
        eng.synchronize()
        q.put((rank, (status, sel.cpu().numpy(), sc.cpu().numpy(), c0, mean.cpu().numpy(),
                      U.cpu().numpy(), X.cpu().numpy())))
        eng.close()
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _run(fail_rank=None, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    return res


needs2 = pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (RCCL ranks)")


@needs2
def test_split_scoring_over_rccl_matches_unsplit(engine):
    from biscotti_amd import _lib
    res = _run()
    U = res[0][5] + res[1][5]  # the 2-rank all-reduce's sum
    Ud = torch.from_numpy(U).cuda()
    Xfull = np.concatenate([res[r][6] for r in (0, 1)], axis=1)
    Xd = torch.from_numpy(Xfull).cuda()
    sel = torch.empty(N - F, dtype=torch.int64, device="cuda")
    sc = torch.empty(N, dtype=torch.float64, device="cuda")
    engine.finish_ptr(Ud.data_ptr(), Xd.data_ptr(), _lib.BK_F64, N, D, D, F, sel.data_ptr(),
                      sc.data_ptr())
    engine.synchronize()
    want_sel, want_sc = sel.cpu().numpy(), sc.cpu().numpy()
    for r in (0, 1):
        status, s, scr, c0, mean, _, Xs = res[r]
        assert status == 0
        assert np.array_equal(s, want_sel), r
        assert np.array_equal(scr.view(np.int64), want_sc.view(np.int64)), r
        ref = Xs[want_sel].mean(axis=0)
        scale = np.max(np.abs(Xs[want_sel]).sum(axis=0) / len(want_sel))
        assert np.max(np.abs(mean - ref)) <= 1e-9 * scale


@needs2
@pytest.mark.parametrize("fail_rank", [0, 1])
def test_failed_share_over_rccl_invalidates_every_rank(fail_rank):
    from biscotti_amd import _lib
    res = _run(fail_rank=fail_rank)
    for r in (0, 1):
        status = res[r][0]
        want = _lib.BK_EHIP if r == fail_rank else _lib.BK_ERCCL
        assert status == want, (r, status)
