"""bench.py's N > 1 orchestration, run once before the driver's 8-GPU run
(VERDICT r2, next-round item 5a): torchrun starts 2 ranks as fresh child
processes on the one MI355X.  RCCL cannot put two ranks on one device, so the
packed partial Grams are summed through gloo on the host (--exchange host:
bk_gram_upper_device -> all_reduce -> bk_finish_device, the decomposition
libbk's RCCL exchange runs).  Covered: the rank bootstrap, the barrier +
max-over-ranks timing, each rank's column shard (synthesised on the device),
the parity of the shard against the reference golden, and the selected-set
hash gathered from every rank."""
import json
import os
import socket
import subprocess
import sys

import pytest

import golden_util as GU

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("workload", [w for w in ("C_1024x131072", "D_512x1M_f256") if GU.have(w)])
def test_bench_two_ranks_host_exchange(workload):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--exchange", "host",
           "--workload", workload, "--no-cpu-baseline", "--no-e2e", "--no-next-rows",
           "--no-graph-probe", "--no-variants"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    # rank 0 prints ONE line and nothing else reaches stdout (library banners
    # such as RCCL's version block go to stderr)
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3
    assert out["config"]["d_local"] < out["config"]["d"]  # rank 0 holds a column shard
    assert out["parity"]["selected_set"] == "match", out["parity"]
    assert out["parity"]["mean"] == "match", out["parity"]  # the shard's sampled columns
    assert not out["parity"]["margin"]["near_tie"]
    assert out["rccl"]["nranks"] == 2 and out["rccl"]["ranks_agree"], out["rccl"]
    assert out["value"] > 0 and out["ms_per_step"] > 0


def test_bench_launches_its_own_ranks():
    """a plain `python3 bench.py --gpus 2` (no torchrun, no
    WORLD_SIZE) starts its own two ranks as a child torch.distributed.run and
    relays rank 0's line: n_gpus 2, both ranks agree on the set, the shard's
    golden matches, and every rank's K1 and exchange time per step are in the
    line, with the replicas form (each rank the whole batch, golden on every
    rank).  The host exchange lets the two ranks share the box's one GPU."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--exchange", "host", "--workload", "C_1024x131072", "--no-cpu-baseline", "--no-e2e",
           "--no-next-rows", "--no-graph-probe"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["parity"]["selected_set"] == "match", out["parity"]
    rc = out["rccl"]
    assert rc["nranks"] == 2 and rc["ranks_agree"], rc
    assert [p["rank"] for p in rc["per_rank"]] == [0, 1]
    assert all(p["k_gram_ms"] > 0 and p["exchange_ms"] > 0 for p in rc["per_rank"]), rc
    assert rc["exchange_ms"] == max(p["exchange_ms"] for p in rc["per_rank"])
    assert sum(p["d_local"] for p in rc["per_rank"]) == out["config"]["d"]
    # the replicas form: each rank the whole batch, no exchange
    rep = out["summary"]["C_1024x131072_replicas"]
    assert rep["sel"] == "match" and rep["value"] > 0, rep


def test_launcher_gpu_count_matches_the_runtime():
    """bench.py's launcher counts GPUs from the KFD topology / visibility
    variables without any GPU runtime; on the GPU box it
    must see exactly the devices the HIP runtime does."""
    sys.path.insert(0, REPO)
    import bench
    import torch
    assert bench.visible_gpus() == torch.cuda.device_count()


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """With the RCCL exchange every rank needs its own GPU: `--gpus N` with
    fewer visible GPUs exits non-zero instead of measuring one GPU."""
    import torch
    have = torch.cuda.device_count()
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", str(have + 1), "--steps", "2", "--warmup", "1",
           "--workload", "C_1024x131072", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not r.stdout.strip(), (r.returncode, r.stdout[-500:])
    assert "visible" in r.stderr


def test_bench_stdout_is_one_json_line_with_rccl():
    """The driver parses bench.py's stdout: with RCCL initialised (the sharded
    path at one rank, as every rank of the 8-GPU run initialises it) RCCL
    prints its version block to fd 1; bench.py sends that to stderr, so
    stdout holds exactly the one JSON line."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "bench.py", "--sharded", "--steps", "2", "--warmup", "1",
           "--workload", "C_1024x131072", "--no-cpu-baseline", "--no-e2e", "--no-next-rows",
           "--no-graph-probe", "--no-variants"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["rccl"]["nranks"] == 1 and out["parity"]["selected_set"] == "match"
