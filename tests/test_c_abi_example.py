"""The C ABI from a plain C caller (examples/krum_cli.c, gcc, no Python in the
process): the call sequence of the cgo shim for getTopKRUMIndex
(DistSys/krum.go:100-166).  CPU: it links against libbk.so and reports
argument errors through bk_last_error.  GPU: its selected set equals the
oracle's."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "examples", "krum_cli")


@pytest.fixture(scope="module")
def cli():
    import __graft_entry__ as G
    G.build_examples()
    return CLI


def test_c_caller_links_and_reports_errors(cli, tmp_path):
    p = tmp_path / "x.bin"
    np.zeros((10, 25)).tofile(p)
    r = subprocess.run([cli, str(p), "10", "25", "0"], capture_output=True, text=True)
    assert r.returncode == 1 and "f < n" in r.stderr  # the reference's f = 0 ValueError
    r = subprocess.run([cli], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,f", [(10, 25, 2), (100, 7850, 50), (129, 4097, 64)])
def test_c_caller_matches_oracle(cli, oracle, tmp_path, n, d, f):
    X = oracle.synth(n, d, 900 + n, f)
    p = tmp_path / "x.bin"
    X.astype("<f8").tofile(p)
    r = subprocess.run([cli, str(p), str(n), str(d), str(f)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split()
    assert lines[0] == "m=%d" % (n - f)
    sel = np.array([int(x) for x in lines[1:]], dtype=np.int64)
    assert np.array_equal(sel, oracle.krum(X, f)[0])
    assert "near_tie=0" in r.stderr, r.stderr  # separated synthetic batches: certified
