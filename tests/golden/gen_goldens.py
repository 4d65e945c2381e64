"""Generate golden vectors by running the REFERENCE Multi-Krum on repo-owned inputs.

Run once in the build container (the only place /root/reference exists):

    python tests/golden/gen_goldens.py [--small-only] [--only NAME ...]

It imports /root/reference/ML/code/logistic_validator.py (the numpy ``krum`` /
``get_krum_scores`` that DistSys/krum.go:100-166 calls through go-python),
with a stub ``utils`` module because the module body loads a dataset that is
not shipped (logistic_validator.py:6-7; .MISSING_LARGE_BLOBS).  Nothing from
the reference is copied: only its outputs on our inputs are saved, as .npz
fixtures (numeric arrays only, loaded with allow_pickle=False) plus
cases.json.

Saved per case:
  sel            sorted(krum(X, f))             -- logistic_validator.py:36-49
  good_idx       krum's raw argpartition order
  scores         get_krum_scores(X, n - f)      -- logistic_validator.py:54-65
  sq             np.sum(X**2, axis=1)           -- :59
  mean / mean_cols+mean_vals, mean_block_sums
                 np.mean(X[good_idx], axis=0)   -- :51 (commented-out aggregate)
  gap            sorted(scores)[m] - sorted(scores)[m-1] (boundary margin)
"""
import argparse
import contextlib
import importlib.util
import io
import json
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import cases as C  # noqa: E402
import synth_np  # noqa: E402

REF = "/root/reference/ML/code/logistic_validator.py"


def load_reference():
    stub = types.ModuleType("utils")
    stub.load_dataset = lambda name: {"X": np.zeros((1, 25)), "y": np.zeros(1)}
    sys.modules["utils"] = stub
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("ref_logistic_validator", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def build_input(p):
    dt = np.float32 if p["dtype"] == "float32" else np.float64
    n, d = p["n"], p["d"]
    if n * d <= 4_000_000:
        X = synth_np.synth(n, d, p["seed"], p["nbyz"], p["mu_scale"], p["byz_scale"],
                           p["sigma"], p["flags"], dtype=dt)
    else:
        # large: the C restatement of the same spec (bit-identical; spot-checked here)
        from oracle import oracle as O
        X = O.synth(n, d, p["seed"], p["nbyz"], p["mu_scale"], p["byz_scale"], p["sigma"],
                    p["flags"], dtype=dt)
        rng = np.random.default_rng(0)
        c0 = int(rng.integers(0, d - 256))
        chk = synth_np.synth(n, d, p["seed"], p["nbyz"], p["mu_scale"], p["byz_scale"],
                             p["sigma"], p["flags"], dtype=dt, c0=c0, dl=256)
        assert np.array_equal(chk.view(np.uint8), X[:, c0:c0 + 256].view(np.uint8)), \
            "numpy and C generators disagree"
    return C.apply_mods(X, p["mods"])


def run_case(ref, name, p, outdir):
    X = build_input(p)
    X64 = X.astype(np.float64)  # exact widening for fp32 inputs
    n, d, f = p["n"], p["d"], p["f"]
    rec = {"name": name, "params": {k: v for k, v in p.items()}}
    if p["error"]:
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                ref.krum(X64, f)
            rec["error"] = None
        except Exception as e:  # the reference raises (argpartition kth out of bounds)
            rec["error"] = type(e).__name__
        return rec
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        good_idx = np.asarray(ref.krum(X64, f))
    t_krum = time.time() - t0
    m = n - f
    scores = ref.get_krum_scores(X64, m)
    sq = np.sum(X64 ** 2, axis=1)
    mean = np.mean(X64[good_idx], axis=0)
    srt = np.sort(scores)
    gap = float(srt[m] - srt[m - 1]) if m < n else float("inf")
    arrays = dict(sel=np.sort(good_idx).astype(np.int64), good_idx=good_idx.astype(np.int64),
                  scores=scores, sq=sq)
    absmean = np.zeros(d)
    for i in np.sort(good_idx):
        absmean += np.abs(X64[i])
    absmean /= m
    rec["mean_scale"] = float(np.nanmax(absmean)) if np.any(np.isfinite(absmean)) else float("nan")
    if d <= C.MEAN_FULL_MAX_D:
        arrays["mean"] = mean
    else:
        cols = C.sample_cols(d, p["seed"])
        arrays["mean_cols"] = cols
        arrays["mean_vals"] = mean[cols]
    bs, edges = C.mean_blocks(mean)
    arrays["mean_block_sums"] = bs
    arrays["mean_block_edges"] = edges
    if n <= 128:
        arrays["D"] = (sq[:, None] + sq[None] - 2 * np.dot(X64, X64.T))
    np.savez_compressed(os.path.join(outdir, name + ".npz"), **arrays)
    rec.update(m=m, gap=gap, max_score=float(np.nanmax(np.abs(scores))) if np.any(np.isfinite(scores)) else None,
               ref_seconds=t_krum, numpy=np.__version__)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small-only", action="store_true")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    ref = load_reference()
    manifest_path = os.path.join(HERE, "cases.json")
    manifest = json.load(open(manifest_path)) if os.path.exists(manifest_path) else {}
    for name in C.CASES:
        p = C.case_params(name)
        if a.only and name not in a.only:
            continue
        if a.small_only and p["large"]:
            continue
        t = time.time()
        manifest[name] = run_case(ref, name, p, HERE)
        print("%-22s %.1fs %s" % (name, time.time() - t,
                                  {k: manifest[name].get(k) for k in ("m", "gap", "error")}), flush=True)
        with open(manifest_path, "w") as fh:
            json.dump(manifest, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
