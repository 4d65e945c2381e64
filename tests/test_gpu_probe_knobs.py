"""The product libbk.so ignores every probe knob.

BK_GRAM_MODE=1 / BK_K2_MODE=1 select timing-only ablations (loads without
MFMAs, keys without the sort) that return a wrong Gram or wrong scores; the
planner overrides (BK_PLAN_*), kernel-shape knobs and traces change how the
same arithmetic is scheduled.  They exist only in -DBK_PROBES builds
(tools/probe_build.py).  A fresh child process sets all of them BEFORE any GPU
call and runs config C (1024 x 131,072, the reference golden) through the
product library: the selection, scores and sampled mean must match the
golden, exactly as without the knobs (reference arithmetic:
ML/code/logistic_validator.py:59-63)."""
import json
import os
import subprocess
import sys

import pytest

pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

KNOBS = {"BK_GRAM_MODE": "1", "BK_K2_MODE": "1", "BK_PLAN_MODE": "0", "BK_PLAN_ROUNDS": "16",
         "BK_PLAN_NB_COST": "9", "BK_QUAD_BAL": "0", "BK_K2_KPT": "4",
         "BK_K2_TRANSPOSE_MIN_N": "1", "BK_SCORES": "v1", "BK_GRAM": "v1",
         "BK_RONI_TILES": "3", "BK_RONI_VALU": "1"}

CHILD = r"""
import json, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
sys.path.insert(0, sys.argv[1] + "/tests/golden")
import golden_util as GU
from biscotti_amd import _lib
from biscotti_amd.krum import Engine
name = "C_1024x131072"
p = GU.C.case_params(name)
n, d, f = p["n"], p["d"], p["f"]
e = Engine(0)
X = torch.empty((n, d), dtype=torch.float64, device="cuda")
e.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, p["seed"], p["nbyz"], p["mu_scale"],
                 p["byz_scale"], p["sigma"], p["flags"])
sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
sc = torch.empty(n, dtype=torch.float64, device="cuda")
mn = torch.empty(d, dtype=torch.float64, device="cuda")
e.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(), sc.data_ptr(),
                       mn.data_ptr())
e.synchronize()
g = GU.load(name)
sel, sc, mn = sel.cpu().numpy(), sc.cpu().numpy(), mn.cpu().numpy()
assert np.array_equal(sel, g["sel"]), "selection differs"
GU.check_scores(sc, g, rel=1e-9)
GU.check_mean(mn, g, GU.manifest()[name])
e.close()
print(json.dumps({"ok": True, "lib": _lib.LIB_PATH}))
"""


def test_probe_knobs_do_not_reach_the_product():
    env = dict(os.environ)
    env.update(KNOBS)
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["lib"].endswith(os.path.join("biscotti_amd", "libbk.so"))
