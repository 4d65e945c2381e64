"""The error paths of libbk on an MI355X (VERDICT r2 "silent-failure and hang
hazards"): an invalid call must say so on the data path and through
every synchronous entry, and no rank may strand its peers in a collective.

Each case runs in a child process, because the knobs are read when a context
is created (bk_create):

* BK_SMALL_SPIN_MAX=<polls>,<launches>: k_small's hand-off waits give up after
  <polls> polls for the next <launches> launches.  At config B the S items'
  workgroups wait for the G phase (~8 us), so one poll always times out.
  bk_multikrum_device returns BK_OK (asynchronous), every selected index is
  -1, bk_synchronize and bk_selection_margin return BK_EHIP, the synchronous
  host entry returns BK_EHIP itself -- and the next launch on the same
  context (same queue counters) is valid again and matches a clean context.
* BK_SMALL_CHECK_LINES=1: the last workgroup out checks that no queue word
  but word 0 of its line was ever written (the invariant the reset relies on,
  bk_small.hip) over launches of alternating shapes.
* BK_TEST_FAIL_BEFORE_EXCHANGE=1|2: a sharded call fails before its exchange
  -- at its signature's status agreement (1) or in steady state (2, the
  partial is poisoned and the rank still joins the exchange).  RCCL at one
  rank (two ranks cannot share one device); the two-rank poisoning through
  the decomposed entries is in tests/test_gpu_two_process.py.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import golden_util as GU

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = r"""
import json, os, sys
sys.path.insert(0, %r)
sys.path.insert(0, os.path.join(%r, "tests", "golden"))
import numpy as np
import torch
from biscotti_amd import _lib
from biscotti_amd.krum import Engine
from oracle import oracle as O

def status_of(fn):
    try:
        fn()
        return 0
    except _lib.BKError as e:
        return e.status
    except ValueError:
        return _lib.BK_EINVAL
""" % (REPO, REPO)


def run_child(body, env, timeout=180):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", PRELUDE + body], env=e, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_small_handoff_timeout_is_reported_everywhere():
    out = run_child(r"""
n, d, f = 100, 7850, 30
X = O.synth(n, d, 20261017, 30, flags=1)
Xd = torch.from_numpy(X).cuda()
eng = Engine(0)
sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
res = {}
# launch 1 (forced timeout): asynchronous entry, then the checks
eng.multikrum_device_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr())
res["sync"] = status_of(eng.synchronize)
res["sel_all_minus1"] = bool((sel.cpu() == -1).all())
res["margin"] = status_of(eng.selection_margin)
# launch 2 (forced timeout): the synchronous host entry reports it itself
res["host"] = status_of(lambda: eng.multikrum(X, f))
# launch 3: the knob is spent -- the same queue counters, a valid call
s3, sc3, m3 = eng.multikrum(X, f)
os.environ.pop("BK_SMALL_SPIN_MAX")  # a clean context to compare with
ref = Engine(0)
s4, sc4, m4 = ref.multikrum(X, f)
res["recovered"] = bool(np.array_equal(s3, s4) and np.array_equal(m3.view(np.int64), m4.view(np.int64)))
res["recovered_sync"] = status_of(eng.synchronize)
osel, _, _ = O.krum(X, f)
res["golden"] = bool(np.array_equal(s3, osel))
print(json.dumps(res))
""", {"BK_SMALL_SPIN_MAX": "1,2"})
    assert out["sync"] == -3, out          # BK_EHIP from bk_synchronize
    assert out["sel_all_minus1"], out      # the data path says so too
    assert out["margin"] == -3, out
    assert out["host"] == -3, out          # bk_multikrum returns it
    assert out["recovered"] and out["recovered_sync"] == 0 and out["golden"], out


def test_small_queue_lines_keep_their_invariant():
    out = run_child(r"""
eng = Engine(0)
ok = True
shapes = [(100, 7850, 30), (50, 3001, 10), (128, 32768, 38), (17, 129, 5), (100, 7850, 30), (3, 300, 1)]
for rep in range(3):
    for (n, d, f) in shapes:
        X = O.synth(n, d, 7 + n, f)
        sel, _, mean = eng.multikrum(X, f)   # checks the margin's codes (BK_EHIP on a dirty line)
        osel, _, _ = O.krum(X, f)
        ok &= bool(np.array_equal(sel, osel))
print(json.dumps({"ok": ok, "sync": status_of(eng.synchronize)}))
""", {"BK_SMALL_CHECK_LINES": "1"})
    assert out == {"ok": True, "sync": 0}


def test_sharded_failure_before_exchange_one_rank():
    out = run_child(r"""
from biscotti_amd.dist import bootstrap_rccl
n, d, f = 200, 4096, 60
X = O.synth(n, d, 5, 40)
Xd = torch.from_numpy(X).cuda()
sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
res = {}
# 1: the status agreement of the signature's first call fails -> error, no exchange
os.environ["BK_TEST_FAIL_BEFORE_EXCHANGE"] = "1"
e1 = Engine(0)
bootstrap_rccl(e1, 0, 1, lambda b, src: b)
res["agree"] = [status_of(lambda: e1.multikrum_sharded_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr())) for _ in range(2)]
res["agree_exchanges"] = e1.comm_stats()[0]
# 2: steady state: the first call agrees and succeeds, the next one fails,
#    poisons its partial, joins the exchange, and the record says invalid
os.environ["BK_TEST_FAIL_BEFORE_EXCHANGE"] = "2"
e2 = Engine(0)
bootstrap_rccl(e2, 0, 1, lambda b, src: b)
e2.multikrum_sharded_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr())
res["first"] = status_of(e2.synchronize)
osel, _, _ = O.krum(X, f)
res["first_golden"] = bool(np.array_equal(sel.cpu().numpy(), osel))
res["steady"] = status_of(lambda: e2.multikrum_sharded_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr()))
res["steady_sync"] = status_of(e2.synchronize)
res["steady_exchanges"] = e2.comm_stats()[0]
print(json.dumps(res))
""", {})
    assert out["agree"] == [-2, -2], out      # BK_ENOMEM (the forced failure), twice, no hang
    assert out["agree_exchanges"] == 0, out   # no data exchange was made
    assert out["first"] == 0 and out["first_golden"], out
    assert out["steady"] == -2, out           # the failing rank's own error
    assert out["steady_sync"] == -4, out      # BK_ERCCL: the poisoned record
    assert out["steady_exchanges"] == 2, out  # it still joined the exchange


def test_group_certified_near_tie_reruns_exact(oracle):
    """bk_group_multikrum honours BK_F32_CERTIFIED.  E_tight
    (4096 x 262,144 fp32, boundary gap 2.8e-12 relative) on G = 2 contexts
    (host exchange, one device): the fp32 MFMA flags the near tie, every
    device re-runs its shard exact, and the group returns the golden set."""
    name = "E_tight_fp32"
    if not GU.have(name):
        pytest.skip("golden not generated")
    from biscotti_amd import _lib
    from biscotti_amd.krum import GroupEngine
    X, p = GU.build_input(name, oracle)
    g = GU.load(name)
    ge = GroupEngine([0, 0], mode=_lib.BK_GROUP_HOST_EXCHANGE)
    try:
        for r in range(2):
            _lib.check(_lib.lib().bk_set_f32_mode(ge.ctx(r), _lib.BK_F32_CERTIFIED))
        r0 = int(_lib.lib().bk_certified_reruns(ge.ctx(0)))
        sel, sc, mean = ge.multikrum(X, p["f"])
        assert np.array_equal(sel, g["sel"])
        assert int(_lib.lib().bk_certified_reruns(ge.ctx(0))) - r0 == 1
        GU.check_mean(mean, g, GU.manifest()[name])
    finally:
        ge.close()
    del X
