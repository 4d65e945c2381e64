"""The premise of K7/K8's bit-exact parity: a chain of
v_mfma_f64_16x16x4_f64 over k ascending rounds exactly like the fp64 FMA chain
acc = fma(a_k, b_k, acc), k ascending -- on fp32-valued and full fp64 operands,
over a wide exponent range, and on two designed cases (four roundings to even;
left-to-right order).  tools/probe_mfma_order (built by __graft_entry__.build)
compares every element of a 16 x 16 block bit for bit."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PROBE = os.path.join(os.path.dirname(HERE), "tools", "probe_mfma_order")


def test_fp64_mfma_rounds_like_an_fma_chain():
    if not os.path.exists(PROBE):
        pytest.fail("tools/probe_mfma_order not built: run __graft_entry__.build()")
    r = subprocess.run([PROBE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if "mfma==valu_fma" in ln]
    assert len(lines) == 14, r.stdout
    for ln in lines:
        assert "mfma==valu_fma 256/256" in ln and "valu==host 256/256" in ln, ln
        assert "max ulp(mfma,fma) 0" in ln, ln
