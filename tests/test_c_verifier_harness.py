"""examples/verifier_harness: Biscotti's Krum verifier flow (DistSys/krum.go
VerifyUpdateKRUM :227-365, startKRUMDeadlineTimer :178-224, computeScores /
getTopKRUMIndex :77-166, checkIfAccepted :47-73) replayed in C with pthreads
over libbk.so through the cgo shim's exact calls (no Go
toolchain in this image).  Concurrent peers append under krumLock, the
threshold-th arrival runs Multi-Krum and releases the waiters, late arrivals
are stale, the deadline timer runs Krum on a partial batch (n < threshold),
and n = 1 (clip = int(0.5) = 0, the reference's ValueError) rejects everyone.
Every verdict is checked against the oracle on the batch the harness reports."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "examples", "verifier_harness")


@pytest.fixture(scope="module")
def harness():
    import __graft_entry__ as G
    G.build_examples()
    return HARNESS


def sid_of(p):
    return (p * 7919) % 10007


def parse(out):
    iters, peers = {}, {}
    for line in out.splitlines():
        t = line.split()
        if t[0] == "iter":
            kv = dict(x.split("=", 1) for x in t[2:])
            ints = lambda s: [int(v) for v in s.split(",")] if s else []  # noqa: E731
            iters[int(t[1])] = dict(path=kv["path"], n=int(kv["n"]), f=int(kv["f"]),
                                    status=int(kv["status"]), near_tie=int(kv["near_tie"]),
                                    batch=ints(kv["batch"]), accepted=ints(kv["accepted"]),
                                    k_small=int(kv["k_small"]), k_gram=int(kv["k_gram"]))
        elif t[0] == "peer":
            peers.setdefault(int(t[1]), {})[int(t[2])] = t[3]
    return iters, peers


def test_harness_usage(harness):
    r = subprocess.run([harness], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("serial_pack", ["0", "1"])  # bk_multikrum_rows / the pre-r6 pinned pack
def test_verifier_flow_against_oracle(harness, oracle, tmp_path, serial_pack):
    rows, d, thresh = 12, 1000, 8
    X = oracle.synth(rows, d, 4242, 3)
    path = tmp_path / "updates.bin"
    X.astype("<f8").tofile(path)
    # iteration 1: 10 peers, threshold 8 -> threshold path, 2 stale
    # iteration 2: 5 peers -> deadline path on n = 5 (f = 2)
    # iteration 3: 1 peer -> deadline path, n = 1, f = 0 -> BK_EINVAL, rejected
    # iteration 4: exactly 8 peers -> threshold path, nobody stale
    arrivals = [10, 5, 1, 8]
    r = subprocess.run([harness, str(path), str(rows), str(d), str(thresh), "400"]
                       + [str(a) for a in arrivals], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, BK_HARNESS_SERIAL_PACK=serial_pack))
    assert r.returncode == 0, r.stderr
    iters, peers = parse(r.stdout)
    assert sorted(iters) == [1, 2, 3, 4]
    sid_row = {sid_of(p): p for p in range(rows)}
    for k, a in enumerate(arrivals, start=1):
        it = iters[k]
        expect_path = "threshold" if a >= thresh else "deadline"
        assert it["path"] == expect_path, (k, it)
        assert it["n"] == min(a, thresh)
        assert it["batch"] == sorted(it["batch"])  # sorted by SourceID (krum.go:306-308)
        assert set(it["batch"]) <= {sid_of(p) for p in range(a)}
        n = it["n"]
        assert it["f"] == int(0.5 * n)  # krum.go:110
        if n == 1:
            assert it["status"] == -1 and it["accepted"] == []  # reject all
            assert it["k_small"] == it["k_gram"] == 0
        else:
            assert it["status"] == 0
            # the host entry took the k_small / k_tiny path, never K1 (one
            # launch, or the pipelined host entry's G launches + one S+M launch)
            assert it["k_small"] >= 1 and it["k_gram"] == 0, it
            Xb = X[[sid_row[s] for s in it["batch"]]]
            osel, _, _ = oracle.krum(Xb, it["f"])
            assert it["accepted"] == [it["batch"][i] for i in osel], (k, it)
        verdicts = peers[k]
        assert len(verdicts) == a
        for s, v in verdicts.items():
            if s not in it["batch"]:
                assert v == "stale"
            else:
                assert v == ("accepted" if s in it["accepted"] else "rejected"), (k, s, v)
        assert sum(v == "stale" for v in verdicts.values()) == a - n


@pytest.mark.gpu
def test_nodes_agree_like_localtest(harness, oracle, tmp_path):
    """The reference's only integration test (DistSys/localTest.sh:47-87): N
    node processes on one host, then every node's log compared with `cmp`.
    Here four verifier processes share the GPU, each replaying two Krum rounds
    of config B's shape (100 peers x 7,850 fp64, threshold 100: no stale or
    deadline race) through libbk; their logs (peer lines in a fixed order) must
    be byte-identical, and the accepted set the oracle's."""
    rows, d = 100, 7850
    X = oracle.synth(rows, d, 20261017, 30)
    path = tmp_path / "updates.bin"
    X.astype("<f8").tofile(path)
    cmd = [harness, str(path), str(rows), str(d), str(rows), "2000", str(rows), str(rows)]
    procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for _ in range(4)]
    logs = []
    for p in procs:
        out, err = p.communicate(timeout=120)
        assert p.returncode == 0, err
        logs.append("\n".join(sorted(out.splitlines())))
    assert all(lg == logs[0] for lg in logs[1:])
    iters, _ = parse(logs[0])
    sid_row = {sid_of(p): p for p in range(rows)}
    for k in (1, 2):
        it = iters[k]
        assert it["path"] == "threshold" and it["n"] == rows and it["status"] == 0
        Xb = X[[sid_row[s] for s in it["batch"]]]
        osel, _, _ = oracle.krum(Xb, it["f"])
        assert it["accepted"] == [it["batch"][i] for i in osel]
