#!/usr/bin/env python3
"""Multi-Krum throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
    torchrun --nproc-per-node N ... bench.py --gpus N     (one rank per GPU)

One step = one full Multi-Krum pass of the hot path over one synthetic batch
already resident in HBM: fp64-MFMA Gram (+ RCCL all-reduce of the packed
partial Gram when N > 1) -> distance rows -> per-row sort and sum of the
n-f-2 nearest -> selection of the n-f lowest -> masked mean.  The default
workload is BASELINE.json's headline config, 512 fp64 updates x 1,048,576
dims, f = 153, with the dimension sharded over the N
ranks (strong scaling: the batch is fixed, each rank owns d/N columns).

value = n * d * 8 bytes / (max-over-ranks wall time per step), in GB/s.
rank 0 prints ONE JSON line; see DESIGN.md "Measurement" for every field.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

SEED0 = 20261015
WORKLOADS = {
    # BASELINE.json configs; D is the headline
    "D_512x1M_f153": dict(n=512, d=1048576, f=153, seed=SEED0 + 4, nbyz=153, dtype="f64"),
    "D_512x1M_f256": dict(n=512, d=1048576, f=256, seed=SEED0 + 4, nbyz=153, dtype="f64"),
    "C_1024x131072": dict(n=1024, d=131072, f=307, seed=SEED0 + 3, nbyz=307, dtype="f64"),
    "B_mnist": dict(n=100, d=7850, f=30, seed=SEED0 + 2, nbyz=30, dtype="f64", flags=1),
    "E_4096x262144_fp32": dict(n=4096, d=262144, f=1228, seed=SEED0 + 5, nbyz=1228, dtype="f32"),
    "A_creditcard": dict(n=10, d=25, f=2, seed=SEED0 + 1, nbyz=2, dtype="f64"),
}
DEFAULT_WORKLOAD = "D_512x1M_f153"
METRIC = "Multi-Krum GB/s (device-resident, n fp64 updates x d) + selected-set parity"
# MI355X dense peaks (MI355X_MICROARCH.md chip table / spec): fp64 matrix 78.6 TF/s,
# fp32 matrix 157.3 TF/s, HBM3E 8 TB/s
PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo; what lscpu prints)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def lib_sha16():
    """the hash PMC records are matched on: libbk.so's device code
    (_lib.code_object_sha16), not the whole file"""
    from biscotti_amd import _lib
    return _lib.code_object_sha16()


def max_over_ranks(v, dev):
    """The max of a host float over the ranks (on the device with RCCL, on the
    host with gloo)."""
    import torch
    import torch.distributed as tdist
    on_dev = tdist.get_backend() == "nccl"
    tt = torch.tensor([v], dtype=torch.float64, device=dev if on_dev else "cpu")
    tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
    return float(tt.item())


def single_call(step, eng, barrier, world, dev, calls=7, idle_s=0.2):
    """What one verifier call sees (krum.go:100-166 runs one Multi-Krum per
    batch): each call starts after >= 150 ms of GPU idle, so the shader clock
    has dropped (DVFS) and the step pays the ramp.  Median over `calls` of the
    whole step (max over ranks) and of K1 (HIP events on libbk's stream)."""
    import torch
    import torch.distributed as tdist
    eng.timing_select(["k_gram", "k_small"])
    steps_ms, k1_ms = [], []
    prev = 0.0
    for _ in range(calls):
        torch.cuda.synchronize()
        barrier()
        time.sleep(idle_s)
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) * 1e3
        if world > 1:
            t = max_over_ranks(t, dev)
        steps_ms.append(t)
        tr = eng.timing_read()
        tot = tr.get("k_gram", tr.get("k_small", {"total_ms": prev}))["total_ms"]
        k1_ms.append(tot - prev)
        prev = tot
    eng.timing_select([])
    return float(np.median(steps_ms)), float(np.median(k1_ms)), steps_ms


def cpu_baseline(w, target_s=10.0, target_1core_s=6.0):
    """Time the oracle (C/OpenMP restatement of the reference's numpy krum,
    oracle/krum_oracle.c) on a bounded sample of the same batch, on all the
    host threads OpenMP is given and on 1 core.  A large
    batch is sampled by columns (its first ds columns, the same n rows); a batch
    whose whole Multi-Krum takes well under the target (configs A and B) is
    run whole, repeatedly, and timed per call."""
    from oracle import oracle as O
    n, d, f = w["n"], w["d"], w["f"]
    dt = np.float32 if w["dtype"] == "f32" else np.float64
    es = 4 if w["dtype"] == "f32" else 8

    def run(ds, reps=1):
        X = O.synth(n, d, w["seed"], w["nbyz"], flags=w.get("flags", 0), dtype=dt, c0=0, dl=ds,
                    d_total=d)
        O.krum(X, f)  # warm (page-in, thread pool)
        t0 = time.perf_counter()
        for _ in range(reps):
            O.krum(X, f)
        return (time.perf_counter() - t0) / reps

    def sized(ds, target):
        t, reps = run(ds), 1
        if t < target / 4 and ds < d:
            ds2 = int(min(d, ds * max(1.0, target / max(t, 1e-3))))
            ds2 = max(8, ds2 // 8 * 8)
            if ds2 > ds:
                ds, t = ds2, run(ds2)
        if ds == d and t < target / 4:  # the whole batch is small: time it per call
            reps = int(min(100000, max(2, target / 2 / max(t, 1e-6))))
            t = run(ds, reps)
        return ds, t, reps

    def what(ds, reps):
        if reps > 1:
            return "the whole %dx%d batch, %d calls" % (n, d, reps)
        return "the first %d of %d columns of the same %dx%d batch" % (ds, d, n, d)

    # first samples of ~2e10 (all cores) / ~1.5e9 (1 core) Gram flops, grown to the target
    def start(flops):
        return int(min(d, max(64, flops / (n * n) // 8 * 8)))

    cores = O.num_threads()
    ds, t, reps = sized(start(2e10), target_s)
    out = {"value": round(n * ds * es / t / 1e9, 4), "unit": "GB/s", "cores": cores,
           "cpu_model": cpu_model(), "kind": "port", "ms_per_call": round(t * 1e3, 4),
           "sample": "oracle/krum_oracle.c (OpenMP, %d threads) full Multi-Krum (Gram, sort, "
                     "select, mean) on %s, %.3f s per call" % (cores, what(ds, reps), t)}
    O.set_threads(1)
    try:
        ds1, t1, reps1 = sized(start(1.5e9), target_1core_s)
    finally:
        O.set_threads(cores)
    out["value_1core"] = round(n * ds1 * es / t1 / 1e9, 4)
    out["ms_per_call_1core"] = round(t1 * 1e3, 4)
    out["sample_1core"] = "same, 1 thread, %s, %.3f s per call" % (what(ds1, reps1), t1)
    return out


F32_MODES = {"exact": 0, "mfma": 1, "certified": 2, "i8": 3, "i8_certified": 4,  # bk_f32_mode
             "i8x2": 5, "i8x2_certified": 6}
I8_MODE_NAMES = ("i8", "i8_certified", "i8x2", "i8x2_certified")
# int8 MFMA dense peak (MI355X: 2x the bf16 rate, ~5 POPS; measured 4.90 on
# v_mfma_i32_32x32x32_i8, profiles/r01/ubench_i8.log)
PEAK_I8_TOPS = 5000.0
I8_PRODUCTS = {"i8": 6, "i8_certified": 6,  # K1i8's digit products (bk_i8.hip): weight >= 2^-26
               "i8x2": 3, "i8x2_certified": 3}  # two digits: weight >= 2^-19


def gram_roofline(n, dl, k_ms, dtype, f32_mode, exact_rerun=False):
    """The dominant kernel's roofline for the arithmetic it ran: fp64 MFMA
    (fp64 rows, fp32 rows exact), fp32 MFMA (BK_F32_MFMA / CERTIFIED), int8
    MFMA (BK_F32_I8*: 6 digit products per Gram element, BK_F32_I8X2*: 3;
    achieved in int8 TOPS, plus the fp64-equivalent rate n(n+1) d / t)."""
    flops = n * (n + 1) * dl
    i8 = f32_mode in I8_MODE_NAMES  # fp32 rows (BK_F32_I8*) or fp64 rows (BK_F64_I8*)
    mode = "exact" if exact_rerun or (dtype != "f32" and not i8) else f32_mode
    if mode in I8_MODE_NAMES:
        ops = I8_PRODUCTS[mode] * flops
        ach = ops / (k_ms * 1e-3) / 1e12
        return {"bound": "mfma", "achieved": round(ach, 3), "peak": PEAK_I8_TOPS, "unit": "TOPS (int8)",
                "frac": round(ach / PEAK_I8_TOPS, 4), "ops_per_launch": ops,
                "fp64_equiv_tflops": round(flops / (k_ms * 1e-3) / 1e12, 3),
                "arithmetic": "int8 MFMA (%d exact digit products)" % I8_PRODUCTS[mode]}
    peak = PEAK_TFLOPS["f32" if mode in ("mfma", "certified") else "f64"]
    ach = flops / (k_ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "flops_per_launch": flops,
            "arithmetic": "fp32 MFMA" if mode in ("mfma", "certified") else "fp64 MFMA"}


def pmc_traffic(tag):
    """HBM bytes per launch of the dominant kernel from profiles/pmc_<tag>.json
    (tools/profile.sh -> tools/pmc_summary.py), used only when that record was
    taken with this very libbk.so build (sha256 prefix); otherwise null."""
    path = os.path.join(REPO, "profiles", "pmc_%s.json" % tag)
    if not os.path.exists(path):
        return None, "no profiles/pmc_%s.json" % tag
    try:
        rec = json.load(open(path))
    except Exception as e:  # noqa: BLE001
        return None, "unreadable profiles/pmc_%s.json: %r" % (tag, e)
    if rec.get("libbk_sha16") != lib_sha16():
        return None, "stale: profiles/pmc_%s.json is from another libbk.so build" % tag
    k = rec.get("k_gram") or rec.get("k_small") or {}
    return k.get("hbm_bytes_per_launch"), "profiles/pmc_%s.json (PMC passes of this libbk.so build)" % tag


def workload_tag(name, f32_mode="exact"):
    return name if f32_mode == "exact" else "%s_%s" % (name, f32_mode)


def device_variant(eng, dev, name, f32_mode="exact", steps=20, warmup=5, X=None):
    """One BASELINE config, device-resident, timed by the driver's own run:
    W >= 5 warm-up calls, K timed steps bracketed by synchronize, K1 (or
    k_small) evented live on libbk's stream, the roofline of that kernel
    (MFMA peak of the arithmetic it runs), its hash-matched PMC traffic, the
    whole step against its floor, and parity (selection + mean against the
    reference golden, plus this call's selection margin)."""
    import torch
    from biscotti_amd import _lib
    w = WORKLOADS[name]
    n, d, f = w["n"], w["d"], w["f"]
    m = n - f
    bdt = _lib.BK_F32 if w["dtype"] == "f32" else _lib.BK_F64
    es = 4 if w["dtype"] == "f32" else 8
    own = X is None
    if own:
        X = torch.empty((n, d), dtype=torch.float32 if es == 4 else torch.float64, device=dev)
        eng.synth_fill_ptr(X.data_ptr(), bdt, n, d, X.stride(0), 0, d, w["seed"], w["nbyz"],
                           flags=w.get("flags", 0))
    sel = torch.empty(m, dtype=torch.int64, device=dev)
    sc = torch.empty(n, dtype=torch.float64, device=dev)
    mean = torch.empty(d, dtype=torch.float64, device=dev)

    def step():
        eng.multikrum_device_ptr(X.data_ptr(), bdt, n, d, X.stride(0), f, sel.data_ptr(),
                                 sc.data_ptr(), mean.data_ptr())

    # fp64 rows take the int8 modes through bk_set_f64_mode (K1i8 for fp64 rows)
    set_mode = eng.set_f64_mode if w["dtype"] == "f64" else eng.set_f32_mode
    set_mode(F32_MODES[f32_mode])
    try:
        r0 = eng.certified_reruns()
        for _ in range(max(5, warmup)):
            step()
        torch.cuda.synchronize()
        k1 = "k_small" if n <= 128 else "k_gram"
        eng.timing_select([k1])
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        kt = eng.timing_read().get(k1, {"avg_ms": float("nan")})
        eng.timing_select([])
        mg = eng.selection_margin()
        reruns = eng.certified_reruns() - r0
    finally:
        set_mode(0)
    roof = gram_roofline(n, d, kt["avg_ms"], w["dtype"], f32_mode, exact_rerun=reruns > 0)
    flops = n * (n + 1) * d
    peak = roof["peak"] if roof["unit"] == "TFLOP/s" else PEAK_TFLOPS["f64"]
    traffic, tsrc = pmc_traffic(workload_tag(name, f32_mode))
    bytes_alg = (n + m) * d * es + 8 * d
    t_mx = (roof["ops_per_launch"] / (PEAK_I8_TOPS * 1e12) if "ops_per_launch" in roof
            else flops / (peak * 1e12))
    t_floor = max(t_mx, bytes_alg / (PEAK_HBM_GBS * 1e9)) * 1e3
    par = golden_check(name, sel.cpu().numpy(), mean.cpu().numpy(), 0, d) or {}
    par["margin"] = {"near_tie": mg["near_tie"], "gap": mg["gap"], "err_bound": mg["err_bound"]}
    out = {"n": n, "d": d, "f": f, "m": m, "dtype": w["dtype"], "f32_mode": f32_mode,
           "warmup": max(5, warmup), "steps": steps, "ms_per_step": round(ms, 4),
           "value": round(n * d * es / (ms * 1e-3) / 1e9, 3), "unit": "GB/s",
           "roofline": dict(roof, traffic=traffic, traffic_source=tsrc, kernel=k1,
                            kernel_avg_ms=round(kt["avg_ms"], 4)),
           "step_roofline": {"t_floor_ms": round(t_floor, 4), "frac": round(t_floor / ms, 4)},
           "parity": par}
    if f32_mode in ("certified", "i8_certified", "i8x2_certified"):
        out["certified_reruns"] = reruns
    if f32_mode in I8_MODE_NAMES:
        kb = eng.timing_read()  # (cleared above) the slicing pass, evented once more
        eng.timing_select(["k_slice", "k_reduce"])
        set_mode(F32_MODES[f32_mode])
        try:
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            kb = eng.timing_read()
        finally:
            eng.timing_select([])
            set_mode(0)
        out["k_slice_ms"] = round(kb.get("k_slice", {"avg_ms": float("nan")})["avg_ms"], 4)
        out["k_reduce_ms"] = round(kb.get("k_reduce", {"avg_ms": float("nan")})["avg_ms"], 4)
    if traffic:
        out["roofline"]["traffic_ratio_to_unique_bytes"] = round(traffic / (n * d * es), 3)
    if own:
        del X
    return out


# config E in its multi-GPU form (BASELINE configs[4]: fp32, 8 x MI355X): the
# exact path, the fp32 MFMA the config names, and the certified two-digit int8 Gram
E_SHARD_MODES = ("exact", "mfma", "i8x2_certified")


def sharded_variant(eng, dev, name, f32_mode, nparts, rank, world, barrier, emu, steps=10,
                    warmup=5, exchange_mode=0, line_mode=0):
    """A BASELINE config in its d-sharded multi-GPU form: this
    rank's column shard through libbk's sharded entry (K1 on the shard, the
    RCCL all-reduce of the packed Gram, split scoring at n >= 2049, the local
    mean).  Timed like the headline: warm-up, barrier, K steps, barrier, max
    over ranks; K1 and the exchange evented live on libbk's stream.  With
    emu > 1 (one GPU): rank 0's shard of an emu-rank job, its rate."""
    import hashlib
    import torch
    import torch.distributed as tdist
    from biscotti_amd import _lib
    from biscotti_amd.dist import shard_bounds
    w = WORKLOADS[name]
    n, d, f = w["n"], w["d"], w["f"]
    m = n - f
    bdt = _lib.BK_F32 if w["dtype"] == "f32" else _lib.BK_F64
    es = 4 if w["dtype"] == "f32" else 8
    c0, dl = shard_bounds(d, nparts, rank)
    X = torch.empty((n, max(dl, 1)), dtype=torch.float32 if es == 4 else torch.float64, device=dev)
    eng.synth_fill_ptr(X.data_ptr(), bdt, n, dl, X.stride(0), c0, d, w["seed"], w["nbyz"],
                       flags=w.get("flags", 0))
    sel = torch.empty(m, dtype=torch.int64, device=dev)
    sc = torch.empty(n, dtype=torch.float64, device=dev)
    mean = torch.empty(max(dl, 1), dtype=torch.float64, device=dev)

    def step():
        eng.multikrum_sharded_ptr(X.data_ptr(), bdt, n, dl, X.stride(0), f, sel.data_ptr(),
                                  sc.data_ptr(), mean.data_ptr())

    set_mode = eng.set_f64_mode if w["dtype"] == "f64" else eng.set_f32_mode
    set_mode(F32_MODES[f32_mode])
    # exchange_mode 2: the all-reduce overlapped with the Gram in pieces
    # (bk_comm_set_mode 2); line_mode: the line's own mode, restored after
    eng.comm_set_mode(exchange_mode)
    try:
        r0 = eng.certified_reruns()
        for _ in range(max(5, warmup)):
            step()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        eng.timing_select(["k_gram", "allreduce", "score_gather", "exchange_exposed"])
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kt = eng.timing_read()
        eng.timing_select([])
        eng.timing_enable(True)  # the per-kernel breakdown, an untimed pass
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        kb = eng.timing_read()
        eng.timing_enable(False)
        mg = eng.selection_margin()
        reruns = eng.certified_reruns() - r0
    finally:
        set_mode(0)
        eng.comm_set_mode(line_mode)
    if world > 1:
        el = max_over_ranks(el, dev)
    ms = el / steps * 1e3
    k1 = kt.get("k_gram", {"avg_ms": float("nan")})["avg_ms"]
    roof = gram_roofline(n, dl, k1, w["dtype"], f32_mode, exact_rerun=reruns > 0)
    h = hashlib.sha256(sel.cpu().numpy().tobytes()).hexdigest()[:16]
    hs = [h]
    def avg(kid):
        v = kt.get(kid)
        return round(v["avg_ms"], 4) if v else None
    mine = {"rank": rank, "k_gram_ms": round(k1, 4), "exchange_ms": avg("allreduce"),
            "score_gather_ms": avg("score_gather")}
    if exchange_mode == 2:
        # the all-reduce span (first start -> last end, overlapping the Gram's
        # later pieces) and the part of it left after the last piece
        ex, sp_ = avg("exchange_exposed"), avg("allreduce")
        mine["exchange_exposed_ms"] = ex
        # clamped at 0: at one rank the span IS the exposed part, and the two
        # event pairs differ by their own granularity (a few us)
        mine["overlapped_fraction"] = (round(max(0.0, 1.0 - ex / sp_), 4)
                                       if ex is not None and sp_ else None)
    per_rank = [mine]
    if world > 1:
        hs, per_rank = [None] * world, [None] * world
        tdist.all_gather_object(hs, h)
        tdist.all_gather_object(per_rank, mine)
    if emu:
        par = {"n/a": "emulated rank 0 of %d: 1/%d of the columns" % (emu, emu)}
    else:
        par = golden_check(name, sel.cpu().numpy(), mean[:dl].cpu().numpy(), c0, dl) or {}
        par["margin"] = {"near_tie": mg["near_tie"], "gap": mg["gap"], "err_bound": mg["err_bound"]}
    out = {"n": n, "d": d, "f": f, "m": m, "dtype": w["dtype"], "f32_mode": f32_mode,
           "parallelism": ("emulated rank 0 of %d (1 GPU)" % emu if emu else
                           "d-shard x%d + RCCL all-reduce" % world),
           "d_local": dl, "warmup": max(5, warmup), "steps": steps, "ms_per_step": round(ms, 4),
           "value": round(n * (dl if emu else d) * es / (ms * 1e-3) / 1e9, 3), "unit": "GB/s",
           "roofline": dict(roof, kernel="k_gram", kernel_avg_ms=round(k1, 4)),
           "kernels_ms_avg": {k: round(v["avg_ms"], 5) for k, v in kb.items()},
           "exchange_ms": max((p["exchange_ms"] for p in per_rank if p["exchange_ms"] is not None),
                              default=None),
           "score_gather_ms": max((p["score_gather_ms"] for p in per_rank
                                   if p["score_gather_ms"] is not None), default=None),
           "per_rank": per_rank, "ranks_agree": len(set(hs)) == 1, "parity": par}
    if f32_mode.endswith("certified"):
        out["certified_reruns"] = reruns
    del X
    torch.cuda.empty_cache()
    return out


def replica_variant(eng, dev, name, world, barrier, steps=20, warmup=5):
    """SURVEY §8(e) 'Replicas' -- the reference's own multi-instance pattern
    (N independent verifiers, DistSys/main.go:1680-1682): every rank runs the
    WHOLE batch on its own GPU through the single-GPU entry, no collective in
    the step.  Timed like the headline (barrier, K steps, barrier, max over
    ranks); value = N batches / step time (weak scaling), each rank's
    selection checked against the golden."""
    import hashlib
    import torch
    import torch.distributed as tdist
    from biscotti_amd import _lib
    w = WORKLOADS[name]
    n, d, f = w["n"], w["d"], w["f"]
    m = n - f
    bdt = _lib.BK_F32 if w["dtype"] == "f32" else _lib.BK_F64
    es = 4 if w["dtype"] == "f32" else 8
    X = torch.empty((n, d), dtype=torch.float32 if es == 4 else torch.float64, device=dev)
    eng.synth_fill_ptr(X.data_ptr(), bdt, n, d, X.stride(0), 0, d, w["seed"], w["nbyz"],
                       flags=w.get("flags", 0))
    sel = torch.empty(m, dtype=torch.int64, device=dev)
    mean = torch.empty(d, dtype=torch.float64, device=dev)

    def step():
        eng.multikrum_device_ptr(X.data_ptr(), bdt, n, d, X.stride(0), f, sel.data_ptr(), None,
                                 mean.data_ptr())
    for _ in range(max(5, warmup)):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    el = max_over_ranks(time.perf_counter() - t0, dev) if world > 1 else time.perf_counter() - t0
    ms = el / steps * 1e3
    par = golden_check(name, sel.cpu().numpy(), mean.cpu().numpy(), 0, d) or {}
    oks = [par.get("selected_set")]
    h = hashlib.sha256(sel.cpu().numpy().tobytes()).hexdigest()[:16]
    hs = [h]
    if world > 1:
        oks, hs = [None] * world, [None] * world
        tdist.all_gather_object(oks, par.get("selected_set"))
        tdist.all_gather_object(hs, h)
    del X
    torch.cuda.empty_cache()
    return {"n": n, "d": d, "f": f, "m": m, "replicas": world, "scaling": "weak",
            "parallelism": "%d independent replicas (no collective)" % world,
            "steps": steps, "ms_per_step": round(ms, 4),
            "value": round(world * n * d * es / (ms * 1e-3) / 1e9, 3), "unit": "GB/s",
            "parity": dict(par, every_rank=oks), "ranks_agree": len(set(hs)) == 1}


def host_entry_variant(eng, dev, name, steps=200, warmup=20, single_calls=7, idle_s=0.2):
    """What a Biscotti verifier's own call costs (krum.go:100-166: the batch
    arrives over RPC into host slices): bk_multikrum(BK_HOST_PINNED) from a
    pinned host batch, H2D + Multi-Krum + D2H of sel and mean, synchronous.
    Steady state (back-to-back calls) and single calls after idle (the clock
    ramp), beside the H2D copy alone and the kernel's HIP-event time, with
    parity against the reference golden."""
    import ctypes
    import torch
    from biscotti_amd import _lib
    w = WORKLOADS[name]
    n, d, f = w["n"], w["d"], w["f"]
    m = n - f
    Xd = torch.empty((n, d), dtype=torch.float64, device=dev)
    eng.synth_fill_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, 0, d, w["seed"], w["nbyz"],
                       flags=w.get("flags", 0))
    Xh = torch.empty((n, d), dtype=torch.float64, pin_memory=True)
    Xh.copy_(Xd)
    selh = np.empty(m, dtype=np.int64)
    meanh = np.empty(d, dtype=np.float64)
    mo = ctypes.c_int64(0)
    L = _lib.lib()

    def call():
        _lib.check(L.bk_multikrum(eng.ctx, ctypes.c_void_p(Xh.data_ptr()), _lib.BK_HOST_PINNED,
                                  _lib.BK_F64, n, d, d, f, selh.ctypes.data, ctypes.addressof(mo),
                                  None, meanh.ctypes.data))

    for _ in range(warmup):
        call()
    t0 = time.perf_counter()
    for _ in range(steps):  # no events in the timed loop (each adds host API time)
        call()
    ms = (time.perf_counter() - t0) / steps * 1e3
    # the kernel's and the copy's own times, from a separate evented pass
    eng.timing_select(["k_small", "k_gram", "h2d", "d2h"])
    for _ in range(max(20, steps // 10)):
        call()
    kt = eng.timing_read()
    eng.timing_select([])
    single = []
    for _ in range(single_calls):
        torch.cuda.synchronize()
        time.sleep(idle_s)
        t0 = time.perf_counter()
        call()
        single.append((time.perf_counter() - t0) * 1e3)
    # the copy alone: the same pinned batch to the device, one H2D per call
    for _ in range(5):
        Xd.copy_(Xh, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        Xd.copy_(Xh, non_blocking=True)
        torch.cuda.synchronize()
    h2d_ms = (time.perf_counter() - t0) / steps * 1e3
    kname = "k_small" if "k_small" in kt else "k_gram"
    # k_tiny shares k_small's timing slot (one workgroup for n <= 16, d <= 128)
    klabel = "k_tiny" if kname == "k_small" and n <= 16 and d <= 128 else kname
    par = golden_check(name, selh.copy(), meanh.copy(), 0, d) or {}
    mg = eng.selection_margin()
    par["margin"] = {"near_tie": mg["near_tie"], "gap": mg["gap"], "err_bound": mg["err_bound"]}
    return {"what": "bk_multikrum(BK_HOST_PINNED): H2D of the %dx%d batch + Multi-Krum + sel and "
                    "mean back to the caller's arrays, synchronous (the verifier's call, krum.go:100-166)" % (n, d),
            "n": n, "d": d, "f": f, "steps": steps, "warmup": warmup,
            "ms_per_call": round(ms, 4), "GB_per_s": round(n * d * 8 / (ms * 1e-3) / 1e9, 3),
            "single_call_ms_median": round(float(np.median(single)), 4),
            "single_calls_ms": [round(x, 4) for x in single],
            "h2d_alone_ms": round(h2d_ms, 4),
            "overhead_over_h2d_ms": round(ms - h2d_ms, 4),
            "kernel": klabel, "kernel_avg_ms": round(kt.get(kname, {"avg_ms": float("nan")})["avg_ms"], 4),
            **({"h2d_evented_ms": round(kt["h2d"]["avg_ms"], 4)} if "h2d" in kt else
               {"input": "read by the kernel from the pinned host batch over PCIe (no H2D copy; "
                         "k_tiny, n <= 16 and d <= 128)"}),
            **({"d2h_evented_ms": round(kt["d2h"]["avg_ms"], 4)} if "d2h" in kt else
               {"outputs": "written by the kernel into mapped pinned host memory (no D2H copy)"}),
            "parity": par}


def rows_entry_variant(eng, dev, name, calls=None, thread_sweep=(1, 2, 4, 8)):
    """The verifier's real input path: n SEPARATELY
    allocated host rows (Go's deltas [][]float64, krum.go:100-166) -> result.
      serial:  the shim's old form -- one thread copies the rows into one
               pinned batch (go/bk/krum_bk.go's copy loop; here np.stack into a
               pinned buffer, a C loop of one memcpy per row), then
               bk_multikrum(BK_HOST_PINNED);
      rows:    bk_multikrum_rows: libbk packs the rows on its host threads into
               a pinned ring, each column chunk's H2D + Gram starting as soon
               as it is packed;
      pinned:  bk_multikrum(BK_HOST_PINNED) on an already-packed batch (the
               e2e_pinned figure: no pack at all), for the ratio.
    Outputs of rows and serial compared bitwise (sel, scores, mean)."""
    import ctypes
    import torch
    from biscotti_amd import _lib
    w = WORKLOADS[name]
    n, d, f = w["n"], w["d"], w["f"]
    m = n - f
    Xd = torch.empty((n, d), dtype=torch.float64, device=dev)
    eng.synth_fill_ptr(Xd.data_ptr(), _lib.BK_F64, n, d, d, 0, d, w["seed"], w["nbyz"],
                       flags=w.get("flags", 0))
    Xh = torch.empty((n, d), dtype=torch.float64, pin_memory=True)
    Xh.copy_(Xd)
    del Xd
    torch.cuda.empty_cache()
    Xn = Xh.numpy()
    rows = []
    for i in range(n):  # n separate allocations, as n RPC-decoded slices
        r = np.empty(d, dtype=np.float64)
        r[:] = Xn[i]
        rows.append(r)
    ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rows])
    L = _lib.lib()
    outs = {k: (np.empty(m, dtype=np.int64), np.empty(n), np.empty(d)) for k in ("rows", "serial")}
    mo = ctypes.c_int64(0)

    def pinned_call(o):
        _lib.check(L.bk_multikrum(eng.ctx, ctypes.c_void_p(Xh.data_ptr()), _lib.BK_HOST_PINNED,
                                  _lib.BK_F64, n, d, d, f, o[0].ctypes.data, ctypes.addressof(mo),
                                  o[1].ctypes.data, o[2].ctypes.data))

    def serial_call():
        np.stack(rows, out=Xn)  # the pack: one thread, one memcpy per row
        pinned_call(outs["serial"])

    def rows_call():
        o = outs["rows"]
        _lib.check(L.bk_multikrum_rows(eng.ctx, ptrs, _lib.BK_F64, n, d, f, o[0].ctypes.data,
                                       ctypes.addressof(mo), o[1].ctypes.data, o[2].ctypes.data))

    def pack_only():
        np.stack(rows, out=Xn)

    big = n * d * 8 > (256 << 20)
    calls = calls or (3 if big else 100 if n * d > 1000 else 1000)
    warm = 2 if big else 20

    def best(fn):
        """big batches: min of `calls` single calls; small ones: the best of 5
        back-to-back blocks of `calls` (the box's other tenants share the host:
        a block's mean is noisy, its best of 5 much less so)"""
        for _ in range(warm):
            fn()
        if big:
            ts = []
            for _ in range(calls):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            return min(ts) * 1e3
        blocks = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(calls):
                fn()
            blocks.append((time.perf_counter() - t0) / calls * 1e3)
        return min(blocks)

    res = {"what": "n separate host rows -> selection + mean on the host (krum.go:100-166)",
           "n": n, "d": d, "f": f, "calls": calls,
           "host_threads_default": int(os.environ.get("BK_HOST_THREADS") or
                                       min(8, os.cpu_count() or 1))}
    res["pack_serial_ms"] = round(best(pack_only), 4)
    res["e2e_rows_serial_ms"] = round(best(serial_call), 4)
    res["e2e_pinned_ms"] = round(best(lambda: pinned_call(outs["serial"])), 4)
    eng.set_host_threads(0)
    res["e2e_rows_ms"] = round(best(rows_call), 4)
    sweep = {}
    for t in thread_sweep:
        eng.set_host_threads(t)
        sweep[str(t)] = round(best(rows_call), 4)
    eng.set_host_threads(0)
    res["e2e_rows_ms_by_threads"] = sweep
    rows_call()
    serial_call()
    a, b = outs["rows"], outs["serial"]
    res["bitwise_same_as_serial"] = {
        "sel": bool(np.array_equal(a[0], b[0])),
        "scores": bool(np.array_equal(a[1].view(np.int64), b[1].view(np.int64))),
        "mean": bool(np.array_equal(a[2].view(np.int64), b[2].view(np.int64)))}
    res["rows_over_pinned"] = round(res["e2e_rows_ms"] / res["e2e_pinned_ms"], 4)
    res["serial_over_pinned"] = round(res["e2e_rows_serial_ms"] / res["e2e_pinned_ms"], 4)
    res["GB_per_s_rows"] = round(n * d * 8 / (res["e2e_rows_ms"] * 1e-3) / 1e9, 3)
    par = golden_check(name, a[0].copy(), a[2].copy(), 0, d) or {}
    res["parity"] = par
    del Xh, rows
    return res


# §8(f) row 4: each call's dominant dispatch and, for the latency-bound one,
# its per-workgroup critical path inputs (bench roni_cases' shapes)
RONI_DOMINANT = {"k_roni": "k_roni_sign_reg<1>", "k_roni_softmax": "k_roni_logits",
                 "k_roni_softmax_batches": "k_roni_batch"}


def roni_roofline(name, ms, meta):
    """What binds a §8(f) row 4 kernel, from the rocprofv3
    record of this very libbk.so build (profiles/pmc_roni.json, written by
    tools/roni_pmc_summary.py; ignored when the library hash differs): the
    dominant dispatch's busiest resource (MFMA pipe, VALU, LDS or HBM, as a
    busy fraction) and frac = that fraction, the share of the time the
    binding resource works; for a latency-bound dispatch (every busy fraction
    low, waves parked most of the time) the one-launch floor instead: the
    empty-dispatch floor of the same trace plus the workgroup's critical path,
    and frac = floor / this launch's time."""
    path = os.path.join(REPO, "profiles", "pmc_roni.json")
    dom = RONI_DOMINANT[name]
    out = {"kernel": dom}
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return dict(out, bound=None, note="no profiles/pmc_roni.json")
    if rec.get("libbk_sha16") != lib_sha16():
        return dict(out, bound=None, note="stale: profiles/pmc_roni.json is from another libbk.so")
    k = rec["kernels"].get(dom, {})
    busy = {r: k.get(f) for r, f in (("mfma", "mfma_busy"), ("valu", "valu_busy"),
                                      ("lds", "lds_busy"), ("hbm", "hbm_frac"))}
    out.update({"busy": {r: (round(v, 4) if v is not None else None) for r, v in busy.items()},
                "waves_parked": k.get("wait_frac"), "waves_per_cu": k.get("waves_per_cu"),
                "dispatch_us_profiled": k.get("us_median"), "source": rec.get("source")})
    top, res_ = max(((v, r) for r, v in busy.items() if v is not None), default=(None, None))
    if name == "k_roni_softmax_batches":
        # one workgroup per update (100 of 256 CUs): the floor of one launch is
        # the empty dispatch plus one workgroup's critical path -- its logit
        # chains read x and w (fp32) from LDS, 8 B per FMA on each of the
        # 2 nb C active threads (LDS: 128 B per cycle per CU), and each chain
        # is d_in + 1 dependent FMAs (>= 4 cycles each)
        clk = (k.get("clock_ghz") or 2.1) * 1e9
        lds_cyc = meta["threads"] * (meta["d_in"] + 1) * 8.0 / 128.0
        chain_cyc = (meta["d_in"] + 1) * 4.0
        floor_us = (rec.get("launch_floor_us") or 0.0) + max(lds_cyc, chain_cyc) / clk * 1e6
        out.update({"bound": "latency (one launch)", "floor_us": round(floor_us, 2),
                    "frac": round(floor_us * 1e-3 / ms, 4),
                    "floor": "empty dispatch %.2f us + per-workgroup LDS-fed FMA chain %.2f us"
                             % (rec.get("launch_floor_us") or 0.0,
                                max(lds_cyc, chain_cyc) / clk * 1e6)})
        return out
    out.update({"bound": res_, "unit": "busy fraction of the binding resource", "peak": 1.0,
                "achieved": round(top, 4) if top is not None else None,
                "frac": round(top, 4) if top is not None else None})
    return out


def launch_floor_ms(dev, reps=200):
    """The box's floor for a one-launch kernel, measured as libbk times its
    kernels (two HIP events around each launch): a 1-workgroup torch kernel
    (a 1-element add) between events, averaged -- what an empty launch costs
    on the same clock, the floor a latency-bound single launch approaches;
    and the back-to-back period of the same launch (dispatch throughput)."""
    import torch
    x = torch.zeros(1, device=dev)
    for _ in range(10):
        x.add_(1.0)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        x.add_(1.0)
        b.record()
    torch.cuda.synchronize()
    each = sum(a.elapsed_time(b) for a, b in evs) / reps
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        x.add_(1.0)
    b.record()
    torch.cuda.synchronize()
    return {"evented_each_ms": round(each, 5), "back_to_back_ms": round(a.elapsed_time(b) / reps, 5)}


def roni_cases(eng, dev):
    """SURVEY §8(f) row 4's kernels on bench-sized inputs: {name: (launch,
    algorithmic bytes or None, what)} -- K7 (logistic RONI over a
    creditcard-test-sized set), K8 over the whole set, and K8 with the
    reference's last-mini-batch semantics (tools/roni_probe.py profiles them)."""
    import torch
    runs = {}
    # RONI (§8(f) row 4): a creditcard-test-sized validation set (30% of
    # 284,807 rows, d = 25: utils.py:86-117) scoring 512 updates in one launch
    from biscotti_amd._lib import check, lib
    nv, dr, nr = 85_000, 25, 512
    g2 = torch.Generator(device=dev).manual_seed(5)
    Xv = torch.randn((nv, dr), dtype=torch.float64, device=dev, generator=g2)
    yv = torch.where(torch.randn(nv, dtype=torch.float64, device=dev, generator=g2) > 0, 1.0, -1.0)
    ww = torch.randn(dr, dtype=torch.float64, device=dev, generator=g2)
    dl = torch.randn((nr, dr), dtype=torch.float64, device=dev, generator=g2) * 1e-2
    rs = torch.empty(nr, dtype=torch.float64, device=dev)
    runs["k_roni"] = (lambda: check(lib().bk_roni_device(eng.ctx, Xv.data_ptr(), nv, dr, dr,
                                                         yv.data_ptr(), ww.data_ptr(),
                                                         dl.data_ptr(), nr, dr, rs.data_ptr())),
                      None, "RONI scores of %d updates on a %d x %d validation set "
                            "(logistic_validator.py:22-33)" % (nr, nv, dr),
                      {"flops": 2.0 * nv * (nr + 1) * dr, "updates": nr})  # nv x (n+1) x d
    # the torch-path RONI (K8, the mnist softmax verifier, ML/Pytorch/client_obj.py:100-112):
    # a 6,000-sample shard of 784 fp32 pixels, 10 classes, 100 updates of 7,850
    nvm, dinm, cm, nrm = 6000, 784, 10, 100
    Xm = torch.randn((nvm, dinm), dtype=torch.float32, device=dev, generator=g2)
    ym = torch.randint(0, cm, (nvm,), dtype=torch.int32, device=dev, generator=g2)
    wm = torch.randn(cm * (dinm + 1), dtype=torch.float64, device=dev, generator=g2) * 0.05
    dm = torch.randn((nrm, cm * (dinm + 1)), dtype=torch.float64, device=dev, generator=g2) * 1e-3
    rsm = torch.empty(nrm, dtype=torch.float64, device=dev)
    ntm = torch.empty(2 * nrm + 1, dtype=torch.int32, device=dev)
    runs["k_roni_softmax"] = (
        lambda: check(lib().bk_roni_softmax_device(eng.ctx, Xm.data_ptr(), nvm, dinm, dinm,
                                                   ym.data_ptr(), cm, wm.data_ptr(), dm.data_ptr(),
                                                   nrm, cm * (dinm + 1), rsm.data_ptr(),
                                                   ntm.data_ptr())),
        None, "softmax RONI scores of %d updates (d = %d), every evaluation over the whole "
              "%d x %d fp32 set, %d classes (ML/Pytorch/client_obj.py:100-112 with batch_size "
              ">= nv)" % (nrm, cm * (dinm + 1), nvm, dinm, cm),
        {"flops": 2.0 * nvm * (nrm + 1) * cm * dinm, "updates": nrm})  # nv x (n+1) x C x d_in
    # the reference's own semantics (client.py:136-144): each update's original and
    # after errors on two random last mini-batches of batch_size 10 (honest.go:47)
    nbm = 10
    im = torch.randint(0, nvm, (nrm, 2, nbm), dtype=torch.int64, device=dev, generator=g2)
    runs["k_roni_softmax_batches"] = (
        lambda: check(lib().bk_roni_softmax_batches_device(
            eng.ctx, Xm.data_ptr(), nvm, dinm, dinm, ym.data_ptr(), cm, wm.data_ptr(),
            dm.data_ptr(), nrm, cm * (dinm + 1), im.data_ptr(), nbm, rsm.data_ptr(),
            ntm.data_ptr())),
        nrm * cm * (dinm + 1) * 8 + 2 * nrm * nbm * dinm * 4 + cm * (dinm + 1) * 8,
        "softmax RONI of %d updates (d = %d), each on its two last mini-batches of %d "
        "samples (client.py:136-144)" % (nrm, cm * (dinm + 1), nbm),
        {"flops": 2.0 * 2 * nrm * nbm * cm * dinm, "updates": nrm, "workgroups": nrm,
         "threads": 2 * nbm * cm, "d_in": dinm})
    return runs


def next_rows(eng, X, n, d, sel, m, steps=5):
    """SURVEY.md §8(f) rows 2-4 on the same device-resident batch (HBM-bound):
    block aggregation of the m selected rows into GlobalW (K4'), the
    secure-path quantised int64 sum (K5), and noise application to 128 of the
    updates with k = 2 noise vectors each (K6).  Algorithmic bytes:
    aggregate m*d*8 + 2*d*8; qsum m*d*8 + 2*d*8; noise rows*d*8*(k+2).  Plus the
    RONI verifier (row 4), batched over 512 updates."""
    import torch
    from biscotti_amd import _lib
    dev = X.device
    g = torch.zeros(d, dtype=torch.float64, device=dev)
    s = torch.empty(d, dtype=torch.int64, device=dev)
    sf = torch.empty(d, dtype=torch.float64, device=dev)
    rows, k = 128, 2
    noise = torch.empty((rows * k, d), dtype=torch.float64, device=dev)
    eng.synth_fill_ptr(noise.data_ptr(), _lib.BK_F64, rows * k, d, d, 0, d, 7, 0, 0.0, 0.0, 1e-3)
    out = torch.empty((rows, d), dtype=torch.float64, device=dev)
    runs = {
        "k_aggregate": (lambda: eng.aggregate_device_ptr(X.data_ptr(), _lib.BK_F64, n, d,
                                                         X.stride(0), sel.data_ptr(), m,
                                                         g.data_ptr()),
                        m * d * 8 + 2 * d * 8,
                        "GlobalW += sum of the %d selected rows (honest.go:360-375)" % m),
        "k_qsum": (lambda: eng.quantized_sum_ptr(X.data_ptr(), _lib.BK_F64, n, d, X.stride(0),
                                                 sel.data_ptr(), m, 4, s.data_ptr(),
                                                 sf.data_ptr()),
                   m * d * 8 + 2 * d * 8,
                   "int64(x*1e4) summed over the %d selected rows (kyber.go:698-757)" % m),
        "k_noise": (lambda: eng.noise_apply_ptr(X.data_ptr(), rows, d, X.stride(0),
                                                noise.data_ptr(), k, d, out.data_ptr(), d),
                    rows * d * 8 * (k + 2),
                    "NoisedDelta = Delta + mean of %d noise vectors, %d updates "
                    "(main.go:1524-1537, 1606-1653)" % (k, rows)),
    }
    runs.update(roni_cases(eng, dev))
    res = {}
    for name, spec in runs.items():
        fn, nbytes, what = spec[:3]
        fn()
        torch.cuda.synchronize()
        eng.timing_enable(True)
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        t = eng.timing_read().get("k_roni" if name.startswith("k_roni") else name)
        eng.timing_enable(False)
        ms = t["avg_ms"]
        if name.startswith("k_roni"):  # §8(f) row 4: what binds, from the PMC record
            meta = spec[3]
            fl, nu = meta["flops"], meta["updates"]
            r = {"what": what, "ms": round(ms, 4), "updates_per_s": round(nu / (ms * 1e-3), 1),
                 "fp64_tflops_algorithmic": round(fl / (ms * 1e-3) / 1e12, 3)}
            if nbytes:
                r["bytes"] = nbytes
            r["roofline"] = roni_roofline(name, ms, meta)
            res[name] = r
            continue
        gbs = nbytes / (ms * 1e-3) / 1e9
        res[name] = {"what": what, "ms": round(ms, 4), "bytes": nbytes, "GB_per_s": round(gbs, 1),
                     "roofline": {"bound": "hbm", "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                  "frac": round(gbs / PEAK_HBM_GBS, 4)}}
    del noise, out
    return res


def graph_probe(eng, dev, X, n, d, f, sel, scores, mean, bdt):
    """bk_graph_enable: the same device-resident step eager vs replayed as one
    hipGraph (no per-kernel events in either), on the headline batch and on the
    launch-bound config B (100 x 7,850)."""
    import torch
    from biscotti_amd import _lib

    def timed(fn, steps):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    wb = WORKLOADS["B_mnist"]
    nb, db, fb = wb["n"], wb["d"], wb["f"]
    Xb = torch.empty((nb, db), dtype=torch.float64, device=dev)
    eng.synth_fill_ptr(Xb.data_ptr(), _lib.BK_F64, nb, db, db, 0, db, wb["seed"], wb["nbyz"],
                       flags=wb.get("flags", 0))
    selb = torch.empty(nb - fb, dtype=torch.int64, device=dev)
    scb = torch.empty(nb, dtype=torch.float64, device=dev)
    mb = torch.empty(db, dtype=torch.float64, device=dev)
    cases = {
        "B_100x7850": (lambda: eng.multikrum_device_ptr(Xb.data_ptr(), _lib.BK_F64, nb, db, db, fb,
                                                        selb.data_ptr(), scb.data_ptr(),
                                                        mb.data_ptr()), 300, nb * db * 8,
                       (selb, mb)),
        "D_512x1M_f153": (lambda: eng.multikrum_device_ptr(X.data_ptr(), bdt, n, d, X.stride(0), f,
                                                           sel.data_ptr(), scores.data_ptr(),
                                                           mean.data_ptr()), 10,
                          n * d * X.element_size(), (sel, mean)),
    }
    res = {}
    eng.timing_enable(False)
    for name, (fn, steps, nbytes, outs) in cases.items():
        eng.graph_enable(False)
        t_eager = timed(fn, steps)
        ref = [o.clone() for o in outs]
        eng.graph_enable(True)
        t_graph = timed(fn, steps)
        same = all(torch.equal(o, r) for o, r in zip(outs, ref))
        eng.graph_enable(False)
        res[name] = {"eager_ms": round(t_eager, 4), "graph_ms": round(t_graph, 4),
                     "graph_GB_per_s": round(nbytes / (t_graph * 1e-3) / 1e9, 2),
                     "bitwise_same": bool(same)}
    return res


def small_variant(eng, dev, name="B_mnist", steps=500, warmup=50):
    """Config B (mnist softmax: 100 x 7,850 fp64, f = 30) or A (creditcard:
    10 x 25, f = 2), the shapes Biscotti's verifiers actually
    run, device-resident: the one-launch k_small path (bk_set_small_path,
    default for n <= 128) against the general six-launch chain on the same
    batch; parity against the config's golden."""
    import torch
    from biscotti_amd import _lib
    w = WORKLOADS[name]
    n, d, f = w["n"], w["d"], w["f"]
    m = n - f
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    eng.synth_fill_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, 0, d, w["seed"], w["nbyz"],
                       flags=w.get("flags", 0))
    sel = torch.empty(m, dtype=torch.int64, device=dev)
    sc = torch.empty(n, dtype=torch.float64, device=dev)
    mean = torch.empty(d, dtype=torch.float64, device=dev)

    def step():
        eng.multikrum_device_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr(),
                                 sc.data_ptr(), mean.data_ptr())

    flops = n * (n + 1) * d
    bytes_alg = (n + m) * d * 8 + 8 * d
    t_floor = max(flops / (PEAK_TFLOPS["f64"] * 1e12), bytes_alg / (PEAK_HBM_GBS * 1e9)) * 1e3
    res = {"n": n, "d": d, "f": f, "steps": steps}
    clock = StreamClock(eng, dev)
    for label, on in (("one_launch", True), ("general_chain", False)):
        eng.set_small_path(on)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        clock.start()
        for _ in range(steps):
            step()
        clock.stop()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        if on:
            batch_ms = clock.ms() / steps
        res[label] = {"ms_per_step": round(ms, 5), "GB_per_s": round(n * d * 8 / (ms * 1e-3) / 1e9, 2),
                      "step_roofline": {"t_floor_ms": round(t_floor, 5),
                                        "bound": "hbm" if bytes_alg / PEAK_HBM_GBS > flops / PEAK_TFLOPS["f64"] / 1e3 else "mfma",
                                        "frac": round(t_floor / ms, 4)},
                      "parity": golden_check(name, sel.cpu().numpy(), mean.cpu().numpy(), 0, d)}
        if res[label]["parity"] is not None:
            mg = eng.selection_margin()
            res[label]["parity"]["margin"] = {"near_tie": mg["near_tie"], "gap": mg["gap"],
                                              "err_bound": mg["err_bound"]}
    eng.set_small_path(True)
    # the one kernel of the one-launch path (k_small, or k_tiny at A): its time
    # per launch is the device time of the timed one-launch loop itself (two
    # HIP events on libbk's stream bracketing the back-to-back launches, so it
    # is never more than the step: VERDICT r4 item 3) -- an upper bound of the
    # kernel's duration (the gaps between launches are in it).  Its HBM
    # roofline over the algorithmic bytes of the call (the Gram's read of X
    # and K4's read of the m selected rows, the mean's write) and its
    # hash-matched PMC traffic.  Events around every launch (a pass of its
    # own) are kept as a diagnostic: each pair adds its own overhead.
    eng.timing_select(["k_small"])
    for _ in range(max(50, steps // 5)):
        step()
    kt = eng.timing_read().get("k_small", {})
    eng.timing_select([])
    if batch_ms > 0:
        traffic, tsrc = pmc_traffic(name)
        ach = bytes_alg / (batch_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "achieved": round(ach, 3), "peak": PEAK_HBM_GBS,
                           "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 5), "traffic": traffic,
                           "traffic_source": tsrc, "kernel": "k_tiny" if n <= 16 and d <= 128 else "k_small",
                           "kernel_avg_ms": round(batch_ms, 5),
                           "kernel_timing": "HIP events on libbk's stream bracketing the %d timed "
                                            "back-to-back launches (per launch, gaps included)" % steps,
                           "kernel_avg_ms_evented_each": round(kt["avg_ms"], 5) if kt.get("avg_ms") else None,
                           "bytes_per_launch": bytes_alg}
        if traffic:
            res["roofline"]["traffic_ratio_to_unique_bytes"] = round(traffic / (n * d * 8), 3)
    res["ms_per_step"] = res["one_launch"]["ms_per_step"]
    res["value"] = res["one_launch"]["GB_per_s"]
    del X
    return res


def golden_check(name, sel_host, mean_local, c0, dl):
    path = os.path.join(REPO, "tests", "golden", name + ".npz")
    if not os.path.exists(path):
        return None
    g = np.load(path, allow_pickle=False)
    ok = bool(np.array_equal(np.sort(sel_host), g["sel"]))
    res = {"selected_set": "match" if ok else "MISMATCH"}
    if "mean" in g.files and mean_local is not None and c0 == 0 and dl == len(g["mean"]):
        man = json.load(open(os.path.join(REPO, "tests", "golden", "cases.json")))
        scale = man[name]["mean_scale"]
        err = float(np.max(np.abs(mean_local - g["mean"])))
        res["mean_max_err_rel"] = err / scale
        res["mean"] = "match" if err <= 1e-9 * scale else "MISMATCH"
    if "mean_cols" in g.files and mean_local is not None:
        cols = g["mean_cols"]
        msk = (cols >= c0) & (cols < c0 + dl)
        if msk.any():
            man = json.load(open(os.path.join(REPO, "tests", "golden", "cases.json")))
            scale = man[name]["mean_scale"]
            err = float(np.max(np.abs(mean_local[cols[msk] - c0] - g["mean_vals"][msk])))
            res["mean_max_err_rel"] = err / scale
            res["mean"] = "match" if err <= 1e-9 * scale else "MISMATCH"
    return res


def noised_probe(eng, dev, X, n, d, f, m, k=1):
    """SURVEY §8(f) row 3 at the bench batch: bk_multikrum_noised from pinned
    host Delta + k pinned noise vectors per update (noise added by K6 as the
    rows land), against the same batch noised on the device
    (bk_noise_apply_device + bk_multikrum_device): selection and mean bitwise."""
    import ctypes
    import torch
    from biscotti_amd import _lib
    g = torch.Generator(device=dev).manual_seed(7)
    Nd = torch.randn((n, k, d), dtype=torch.float64, device=dev, generator=g) * 1e-4
    Dh = torch.empty((n, d), dtype=torch.float64, pin_memory=True)
    Dh.copy_(X[:, :d])
    Nh = torch.empty((n, k, d), dtype=torch.float64, pin_memory=True)
    Nh.copy_(Nd)
    selh = np.empty(m, dtype=np.int64)
    meanh = np.empty(d, dtype=np.float64)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        eng.multikrum_noised_ptr(Dh.data_ptr(), d, Nh.data_ptr(), k, d, _lib.BK_HOST_PINNED, n,
                                 d, f, selh.ctypes.data, None, meanh.ctypes.data)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    # reference on the device: noise a resident copy, then the device entry
    Xn = torch.empty((n, d), dtype=torch.float64, device=dev)
    eng.noise_apply_ptr(X.data_ptr(), n, d, X.stride(0), Nd.data_ptr(), k, d, Xn.data_ptr(), d)
    sel2 = torch.empty(m, dtype=torch.int64, device=dev)
    mean2 = torch.empty(d, dtype=torch.float64, device=dev)
    eng.multikrum_device_ptr(Xn.data_ptr(), _lib.BK_F64, n, d, d, f, sel2.data_ptr(), None,
                             mean2.data_ptr())
    torch.cuda.synchronize()
    same_sel = bool(np.array_equal(selh, sel2.cpu().numpy()))
    same_mean = bool(np.array_equal(meanh.view(np.int64), mean2.cpu().numpy().view(np.int64)))
    del Xn, Nd, Dh, Nh
    return {"k": k, "ms": round(t * 1e3, 3),
            "GB_per_s": round(n * d * 8 / t / 1e9, 3),
            "pcie_GB_per_s": round(n * d * 8 * (1 + k) / t / 1e9, 3),
            "selected_set_same": same_sel, "mean_bitwise_same": same_mean}


def _r(x, nd=4):
    return None if x is None else round(float(x), nd)


def _summ(v, host=None):
    """One config's numbers for the compact line's summary: value (GB/s),
    ms_per_step, the dominant kernel's roofline frac, PMC traffic over the
    unique input bytes, selected-set parity and the near-tie flag."""
    roof = v.get("roofline") or {}
    par = v.get("parity") or {}
    if "one_launch" in v:  # small_variant: parity sits with the one-launch timing
        par = dict(v["one_launch"].get("parity") or {}, **{k: x for k, x in par.items()})
    traffic = roof.get("traffic")
    ub = roof.get("unique_bytes")
    s = {"value": v.get("value"), "ms": v.get("ms_per_step"),
         "kernel": roof.get("kernel"), "kernel_ms": roof.get("kernel_avg_ms"),
         "frac": roof.get("frac"), "peak": roof.get("peak"),
         "traffic_ratio": roof.get("traffic_ratio_to_unique_bytes") or
         (_r(traffic / ub, 3) if traffic and ub else None),
         "sel": par.get("selected_set"), "mean": par.get("mean"),
         "near_tie": (par.get("margin") or {}).get("near_tie")}
    if "certified_reruns" in v:
        s["reruns"] = v["certified_reruns"]
    if "error" in v:
        s["error"] = v["error"]
    if "replicas" in v:
        s["replicas"] = v["replicas"]
        s["ranks_agree"] = v.get("ranks_agree")
    if "per_rank" in v:  # a d-sharded variant: the slowest rank's exchange and score gather
        s["exchange_ms"] = v.get("exchange_ms")
        s["score_gather_ms"] = v.get("score_gather_ms")
        ov = [p.get("overlapped_fraction") for p in v["per_rank"] if p]
        if any(x is not None for x in ov):
            s["exposed_ms"] = max((p.get("exchange_exposed_ms") or 0.0) for p in v["per_rank"] if p)
            s["overlapped_fraction"] = min(x for x in ov if x is not None)
    if host:
        s["host_ms"] = host.get("ms_per_call")
        s["host_over_h2d_ms"] = host.get("overhead_over_h2d_ms")
        s["host_sel"] = (host.get("parity") or {}).get("selected_set")
    return s


def compact_line(out, detail_path):
    """The printed JSON line: the contract's keys, the headline's roofline,
    cpu_baseline and parity, and -- as the LAST key -- a per-config summary of
    every BASELINE config measured in this run, so the driver's stored tail
    holds all of them.  The full record goes to
    detail_path (copied under profiles/ for the judged runs)."""
    try:
        os.makedirs(os.path.dirname(detail_path), exist_ok=True)
        with open(detail_path, "w") as fp:
            json.dump(out, fp, indent=1)
    except OSError as e:
        detail_path = "unwritable (%r)" % (e,)
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")
    line = {k: out[k] for k in keep if k in out}
    roof = dict(out["roofline"])
    roof.pop("traffic_source", None)
    line["roofline"] = roof
    cb = out.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample",
                                                    "value_1core", "cpu_model", "error") if k in cb}
    par = out.get("parity")
    if par:
        line["parity"] = par
    for k in ("step_roofline", "rccl"):
        if out.get(k):
            line[k] = out[k]
    line["detail_file"] = os.path.relpath(detail_path, REPO) if os.path.isabs(detail_path) else detail_path
    summ = {}
    head = {"value": out["value"], "ms_per_step": out["ms_per_step"], "roofline": out["roofline"],
            "parity": out.get("parity")}
    tag = out["config"]["workload"]
    if "f32_mode" in out["config"] and out["config"]["f32_mode"] != "exact":
        tag += "_" + out["config"]["f32_mode"]
    summ[tag] = _summ(head)
    for name, v in (out.get("variants") or {}).items():
        summ[name] = _summ(v, v.get("host_entry"))
    sc = out.get("single_call")
    if sc:
        summ["single_call"] = {"ms": sc["ms"], "k_gram_frac": sc.get("k_gram_frac")}
    nr = out.get("next_rows")
    if nr:
        summ["next_rows"] = {k: {"ms": v.get("ms"), "frac": (v.get("roofline") or {}).get("frac")}
                             for k, v in nr.items()}
    e2e = out.get("e2e_pinned_h2d_d2h")
    if e2e:
        summ["e2e_pinned"] = {"GB_per_s": e2e["GB_per_s"], "ms": e2e["ms"]}
    for nm, v in (out.get("e2e_rows") or {}).items():
        summ.setdefault("e2e_rows", {})[nm] = (
            {"error": v["error"]} if "error" in v else
            {"rows_ms": v["e2e_rows_ms"], "serial_ms": v["e2e_rows_serial_ms"],
             "pinned_ms": v["e2e_pinned_ms"], "rows_over_pinned": v["rows_over_pinned"],
             "bitwise": all(v["bitwise_same_as_serial"].values()),
             "sel": (v.get("parity") or {}).get("selected_set")})
    line["summary"] = summ
    return line


class StreamClock:
    """Two HIP events on libbk's own stream (torch.cuda.ExternalStream of
    bk_get_stream) bracketing a batch of back-to-back launches: the device
    time of the batch, never more than the host's wall time around it."""

    def __init__(self, eng, dev):
        import torch
        self.s = torch.cuda.ExternalStream(eng.stream(), device=dev)
        self.a = torch.cuda.Event(enable_timing=True)
        self.b = torch.cuda.Event(enable_timing=True)

    def start(self):
        self.a.record(self.s)

    def stop(self):
        self.b.record(self.s)

    def ms(self):
        self.b.synchronize()
        return float(self.a.elapsed_time(self.b))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpus(environ=None, topology="/sys/class/kfd/kfd/topology/nodes", dri="/dev/dri"):
    """GPUs this process could use, counted with no GPU runtime at all (VERDICT
    r5 item 5): the launcher parent imports neither torch nor HIP and never
    opens /dev/kfd.  A visibility list in the environment decides
    (ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES, then CUDA_VISIBLE_DEVICES,
    as the ROCm runtime applies them: the count of its comma-separated
    entries, an empty list meaning none); otherwise the KFD topology's nodes
    whose gpu_id is non-zero (CPU nodes have gpu_id 0) and whose render node
    (/dev/dri/renderD<drm_render_minor>) this process may open -- the filter
    the ROCm runtime applies in a container that exposes only some GPUs
    (os.access: the node is not opened)."""
    env = os.environ if environ is None else environ
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if var in env:
            v = env[var].strip()
            return len([x for x in v.split(",") if x.strip()]) if v else 0
    count = 0
    try:
        nodes = os.listdir(topology)
    except OSError:
        return 0
    for nd in nodes:
        try:
            with open(os.path.join(topology, nd, "gpu_id")) as fp:
                if int(fp.read().strip() or "0") == 0:
                    continue
        except (OSError, ValueError):
            continue
        minor = None
        try:
            with open(os.path.join(topology, nd, "properties")) as fp:
                for ln in fp:
                    t = ln.split()
                    if len(t) == 2 and t[0] == "drm_render_minor":
                        minor = int(t[1])
        except (OSError, ValueError):
            pass
        if minor is not None and minor > 0:
            node = os.path.join(dri, "renderD%d" % minor)
            if not os.access(node, os.R_OK | os.W_OK):
                continue
        count += 1
    return count


def launch_ranks(a, argv=None, gpus_fn=visible_gpus):
    """`python bench.py --gpus N` without WORLD_SIZE: start N ranks as ONE
    child `python -m torch.distributed.run --nproc-per-node N bench.py ...`
    (a fresh process, never an exec: this parent touches no GPU), relay rank
    0's JSON line to stdout and return the child's exit status.  With the RCCL
    exchange every rank needs a GPU of its own: fewer visible GPUs than N is an
    error (non-zero exit), never a silent 1-GPU measurement.  The host
    exchange (--exchange host) lets ranks share a GPU (the 1-GPU box's test of
    this launcher)."""
    import subprocess
    argv = list(sys.argv[1:] if argv is None else argv)
    have = gpus_fn()
    if a.exchange == "rccl" and have < a.gpus:
        log("bench.py: --gpus %d needs %d GPUs, %d visible; not measuring fewer" % (a.gpus, a.gpus, have))
        return 3
    if have < 1:
        log("bench.py: no GPU visible")
        return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(a.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    log("bench.py: launching %d ranks: %s" % (a.gpus, " ".join(cmd)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    import signal
    p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, text=True)

    def forward(sig, _frame):  # a time limit that signals this parent reaches the ranks too
        p.send_signal(sig)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    lines = []
    for ln in p.stdout:  # rank 0's line (the ranks send everything else to stderr)
        if ln.strip():
            lines.append(ln)
    rc = p.wait()
    for ln in lines:
        if ln.lstrip().startswith("{"):
            sys.stdout.write(ln if ln.endswith("\n") else ln + "\n")
        else:
            log(ln.rstrip("\n"))
    sys.stdout.flush()
    if rc == 0 and not any(ln.lstrip().startswith("{") for ln in lines):
        log("bench.py: the ranks exited 0 without a JSON line")
        return 4
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the GPU clock ramps over the first launches after idle (per-dispatch
    # trace, profiles/r01/rocprof_D_v6.md): warm up past it
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default=DEFAULT_WORKLOAD, choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-next-rows", action="store_true",
                    help="skip the §8(f) aggregation / quantised-sum / noise measurements")
    ap.add_argument("--no-graph-probe", action="store_true",
                    help="skip the eager-vs-hipGraph probe (keeps rocprof per-kernel averages "
                         "to the headline shape)")
    ap.add_argument("--deterministic", action="store_true",
                    help="multi-GPU: all-gather + fixed-order sum instead of all-reduce")
    ap.add_argument("--sharded", action="store_true",
                    help="use the sharded path + RCCL communicator even at 1 rank")
    ap.add_argument("--f32-mode", default="exact", choices=sorted(F32_MODES),
                    help="fp32 workloads (E): exact (fp32 widened onto the fp64 MFMA), mfma "
                         "(the fp32 MFMA), certified (fp32 MFMA, exact re-run on a near tie)")
    ap.add_argument("--no-variants", action="store_true",
                    help="only the workload itself (rocprof PMC passes): no other BASELINE "
                         "configs, modes or host-entry lines")
    ap.add_argument("--exchange", default="rccl", choices=("rccl", "host"),
                    help="N > 1: the packed-Gram exchange inside libbk over RCCL (default), or "
                         "through torch.distributed gloo on the host (bk_gram_upper_device -> "
                         "all_reduce -> bk_finish_device; lets N ranks share one GPU in tests)")
    ap.add_argument("--detail-out", default=os.path.join(REPO, "gpurun_out", "bench_detail.json"),
                    help="where the full record goes (every variant, kernel breakdown, probes); "
                         "the printed line is the compact form with a per-config summary")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="tuning aid on a 1-GPU box: run rank 0's column shard of an N-rank "
                         "job (sharded path, 1-rank RCCL exchange); value is that rank's rate")
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` starts its own N ranks
        sys.exit(launch_ranks(a))
    # the JSON line is the only thing on stdout: libraries that print banners
    # to fd 1 (RCCL's init prints its version block there) are sent to stderr,
    # and the line goes to the saved stdout at the end
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log("note: WORLD_SIZE=%d, --gpus=%d; using WORLD_SIZE" % (world, a.gpus))

    import torch
    import torch.distributed as tdist

    from biscotti_amd import _lib
    from biscotti_amd.dist import bootstrap_rccl, shard_bounds, torch_broadcast_bytes
    from biscotti_amd.krum import Engine

    host_exch = a.exchange == "host" and world > 1
    # one rank per GPU; with the host exchange several ranks may share one
    # (tests run N = 2 on a 1-GPU box)
    dev_idx = local_rank % max(1, torch.cuda.device_count()) if host_exch else local_rank
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    sharded = world > 1 or a.sharded
    if sharded:
        if not tdist.is_initialized() and "MASTER_ADDR" in os.environ:
            if host_exch:
                tdist.init_process_group("gloo")
            else:
                tdist.init_process_group("nccl", device_id=dev)

    w = WORKLOADS[a.workload]
    n, d, f = w["n"], w["d"], w["f"]
    m = n - f
    emu = a.emulate_ranks if world == 1 and a.emulate_ranks > 1 else 0
    if emu:
        sharded = a.sharded = True
    c0, dl = shard_bounds(d, emu or world, rank)
    tdt = torch.float32 if w["dtype"] == "f32" else torch.float64
    bdt = _lib.BK_F32 if w["dtype"] == "f32" else _lib.BK_F64
    es = 4 if w["dtype"] == "f32" else 8

    if emu:
        # split scoring as rank 0 of emu ranks would run it (n >= 2049: config
        # E): its share of K2's rows only, once a mode's first call scored all
        os.environ["BK_EMU_SPLIT_SCORES"] = str(emu)
    eng = Engine(dev_idx)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    # fp64 rows take the int8 modes through bk_set_f64_mode (K1i8 for fp64 rows)
    f64_i8 = w["dtype"] == "f64" and a.f32_mode in I8_MODE_NAMES
    if w["dtype"] == "f64" and a.f32_mode not in ("exact",) + I8_MODE_NAMES:
        raise SystemExit("--f32-mode %s applies to fp32 rows only" % a.f32_mode)
    if f64_i8:
        eng.set_f64_mode(F32_MODES[a.f32_mode])
    else:
        eng.set_f32_mode(F32_MODES[a.f32_mode])
    if sharded and not host_exch:
        if tdist.is_initialized():
            bootstrap_rccl(eng, rank, world, torch_broadcast_bytes)
        else:
            bootstrap_rccl(eng, 0, 1, lambda b, src: b)
        eng.comm_set_mode(a.deterministic)

    X = torch.empty((n, max(dl, 1)), dtype=tdt, device=dev)
    eng.synth_fill_ptr(X.data_ptr(), bdt, n, dl, X.stride(0), c0, d, w["seed"], w["nbyz"],
                       flags=w.get("flags", 0))
    sel = torch.empty(m, dtype=torch.int64, device=dev)
    scores = torch.empty(n, dtype=torch.float64, device=dev)
    mean = torch.empty(max(dl, 1), dtype=torch.float64, device=dev)

    if host_exch:
        usz = int(_lib.lib().bk_upper_elems(n))
        Ud = torch.empty(usz, dtype=torch.float64, device=dev)
        Uh = torch.empty(usz, dtype=torch.float64)
    host_exch_s = [0.0]  # the host exchange's wall time (D2H + gloo all_reduce + H2D)

    def step_f(ff, sel_t):
        if not sharded:
            eng.multikrum_device_ptr(X.data_ptr(), bdt, n, dl, X.stride(0), ff, sel_t.data_ptr(),
                                     scores.data_ptr(), mean.data_ptr())
        elif host_exch:
            # bk_gram_upper_device -> sum over ranks on the host (gloo) -> bk_finish_device:
            # the same decomposition as libbk's RCCL exchange (tests/test_gpu_two_process.py)
            # (libbk runs on its own stream when torch's is the null stream:
            # order the copies explicitly)
            eng.gram_upper_ptr(X.data_ptr(), bdt, n, dl, X.stride(0), Ud.data_ptr())
            eng.synchronize()
            te = time.perf_counter()
            Uh.copy_(Ud)
            tdist.all_reduce(Uh)
            Ud.copy_(Uh)
            torch.cuda.synchronize()
            host_exch_s[0] += time.perf_counter() - te
            eng.finish_ptr(Ud.data_ptr(), X.data_ptr(), bdt, n, dl, X.stride(0), ff,
                           sel_t.data_ptr(), scores.data_ptr(), mean.data_ptr())
        else:
            eng.multikrum_sharded_ptr(X.data_ptr(), bdt, n, dl, X.stride(0), ff, sel_t.data_ptr(),
                                      scores.data_ptr(), mean.data_ptr())

    def step():
        step_f(f, sel)

    def barrier():
        if world > 1:
            tdist.barrier()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    # the roofline kernel (K1; k_small, the one-launch path, for n <= 128) is
    # timed live with HIP events on libbk's stream; the other kernels are not,
    # so the timed region carries no extra events
    # at N > 1 the exchange (libbk's RCCL all-reduce) is evented too: each
    # rank's K1 and exchange time per step go into the line
    # a us-scale one-launch step (k_small, n <= 128) pays two event records as
    # much as it computes: there two events on libbk's stream bracket the
    # whole timed loop instead (per-launch device time, gaps included, never
    # more than the step)
    # (libbk's own predicate for the one-launch path, small_ok: n <= 128, d <=
    # min(32768, BK_SMALL_MAX_D), BK_SMALL not 0 -- any mode: it is always
    # exact; the evented breakdown below confirms which path ran -- ADVICE r5)
    small_step = (not sharded and n <= 128 and os.environ.get("BK_SMALL", "1") != "0" and
                  dl <= min(32768, int(os.environ.get("BK_SMALL_MAX_D") or 32768)))
    eng.timing_select(([] if small_step else ["k_gram"]) +
                      (["allreduce"] if sharded and not host_exch else []))
    tstride = 1
    clock = StreamClock(eng, dev)
    host_exch_s[0] = 0.0
    t0 = time.perf_counter()
    clock.start()
    for _ in range(a.steps):
        step()
    clock.stop()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    kt = eng.timing_read()
    if small_step:
        kt["k_small"] = {"avg_ms": clock.ms() / a.steps, "count": a.steps}
    host_exch_ms = host_exch_s[0] / a.steps * 1e3
    eng.timing_stride(1)
    # per-kernel breakdown from a separate, untimed pass (every kernel evented)
    eng.timing_enable(True)
    for _ in range(max(3, a.steps // 4)):
        step()
    torch.cuda.synchronize()
    kbreak = eng.timing_read()
    eng.timing_enable(False)
    if small_step and "k_small" not in kbreak and "k_gram" in kbreak:
        # the general chain ran after all: its K1 is the roofline kernel (the
        # untimed pass's events), not the loop-bracketed clock
        log("bench.py: n <= 128 but the one-launch path did not run; K1 from the evented pass")
        kt.pop("k_small", None)
        kt["k_gram"] = kbreak["k_gram"]
        small_step = False
    # the selection margin of this batch (bk_selection_margin): near_tie False
    # proves the reference's argpartition selects exactly this set
    mg = eng.selection_margin()
    elapsed = t1 - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)
    ms_per_step = elapsed / a.steps * 1e3
    value = n * (dl if emu else d) * es / (elapsed / a.steps) / 1e9

    EMU_NOTE = {"n/a": "emulated rank: the selection uses 1/%d of the columns, so it is not "
                       "comparable with the full-d golden" % (emu or 1)}
    parity = EMU_NOTE if emu else golden_check(a.workload, sel.cpu().numpy(),
                                                mean[:dl].cpu().numpy(), c0, dl)

    variants = {}
    if a.workload == "D_512x1M_f153" and not a.no_variants:
        # the reference's own clip rule, f = int(0.5 n) (krum.go:110), on the same batch
        f2 = n // 2
        sel2 = torch.empty(n - f2, dtype=torch.int64, device=dev)

        def step2():
            step_f(f2, sel2)
        for _ in range(max(5, a.warmup)):  # its own warm-up (r2's one call under-warmed it)
            step2()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        k2 = max(10, a.steps // 2)
        eng.timing_select(["k_gram"])  # K1 evented live, as on the headline line
        t0 = time.perf_counter()
        for _ in range(k2):
            step2()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        e2 = time.perf_counter() - t0
        kt2 = eng.timing_read().get("k_gram", {"avg_ms": float("nan")})
        eng.timing_select([])
        mg2 = eng.selection_margin()
        if world > 1:
            e2 = max_over_ranks(e2, dev)
        roof2 = gram_roofline(n, dl, kt2["avg_ms"], w["dtype"], a.f32_mode)
        tr2 = None
        if world == 1 and not emu:
            tr2, _ = pmc_traffic(workload_tag(a.workload, a.f32_mode))  # the same K1 launch shape
        par2 = EMU_NOTE if emu else golden_check("D_512x1M_f256", sel2.cpu().numpy(),
                                                 mean[:dl].cpu().numpy(), c0, dl)
        if not emu and par2 is not None:
            par2 = dict(par2, margin={"near_tie": mg2["near_tie"], "gap": mg2["gap"],
                                      "err_bound": mg2["err_bound"]})
        variants["D_512x1M_f256"] = {
            "f": f2, "m": n - f2, "steps": k2, "ms_per_step": round(e2 / k2 * 1e3, 4),
            "value": round(n * (dl if emu else d) * es / (e2 / k2) / 1e9, 3),
            "roofline": dict(roof2, kernel="k_gram", kernel_avg_ms=round(kt2["avg_ms"], 4),
                             traffic=tr2,
                             **({"traffic_ratio_to_unique_bytes": round(tr2 / (n * dl * es), 3)}
                                if tr2 else {})),
            "parity": par2}

    if sharded and not host_exch and not a.no_variants and a.workload == DEFAULT_WORKLOAD:
        # config E at this rank count (BASELINE: fp32, 8 x MI355X), each rank
        # its own column shard, beside the headline D (d-sharded the same way)
        # each mode twice: the exchange after the whole Gram (mode 0), and
        # overlapped with it in pieces (bk_comm_set_mode 2, tag "_overlap":
        # per rank the all-reduce span, its exposed part and the overlapped
        # fraction) -- the driver's N-GPU run decides between them
        line_mode = 1 if a.deterministic else 0
        stop = False
        for mode in E_SHARD_MODES:
            for xm, suffix in ((0, ""), (2, "_overlap")):
                tag = workload_tag("E_4096x262144_fp32", mode) + suffix
                try:
                    variants[tag] = sharded_variant(eng, dev, "E_4096x262144_fp32", mode,
                                                    emu or world, rank, world, barrier, emu,
                                                    exchange_mode=xm, line_mode=line_mode)
                except Exception as e:  # noqa: BLE001 -- a variant's failure must not cost the headline line
                    log("bench.py: sharded variant %s failed: %r" % (tag, e))
                    variants[tag] = {"error": repr(e)}
                    stop = True  # the ranks may no longer be in step: no further collective variants
                    break
            if stop:
                break
    ranks_in_step = True
    if world > 1 and not a.no_variants:
        # every rank learns whether any rank's sharded variant failed before
        # the collectives that follow (replica_variant's barrier and gathers):
        # ranks that disagree about running them would hang
        failed = any("error" in v for v in variants.values() if isinstance(v, dict))
        flag = torch.tensor([1.0 if failed else 0.0], dtype=torch.float64,
                            device=dev if not host_exch else "cpu")
        tdist.all_reduce(flag, op=tdist.ReduceOp.MAX)
        ranks_in_step = float(flag.item()) == 0.0
        if not ranks_in_step:
            log("bench.py: a rank's sharded variant failed; skipping the replica variant")
    if world > 1 and not a.no_variants and WORKLOADS[a.workload]["n"] > 128 and ranks_in_step:
        # the reference's own scale-out: N independent verifiers, one batch each
        # (no exchange, so it runs under --exchange host too)
        variants[a.workload + "_replicas"] = replica_variant(eng, dev, a.workload, world, barrier)

    # roofline of the dominant kernel (K1, fp64 MFMA): algorithmic flops per
    # launch = n(n+1) * d_local (symmetric Gram incl. diagonal)
    k1name = "k_gram" if "k_gram" in kt else "k_small"
    g = kt.get(k1name, {"avg_ms": float("nan")})
    flops = n * (n + 1) * dl
    # fp64 rows and exact fp32 rows (widened) run the fp64 MFMA; BK_F32_MFMA /
    # CERTIFIED the fp32 MFMA; BK_F32_I8* the int8 MFMA
    groof = gram_roofline(n, dl, g["avg_ms"], w["dtype"], a.f32_mode)
    peak = groof["peak"] if groof["unit"] == "TFLOP/s" else PEAK_TFLOPS["f64"]
    # traffic: HBM bytes per K1 launch from the rocprofv3 PMC passes
    # (tools/profile.sh -> tools/pmc_summary.py), used only when that record was
    # taken with this very libbk.so build (sha256 prefix); otherwise null
    traffic, traffic_src = None, None
    if world == 1 and not emu:
        traffic, traffic_src = pmc_traffic(workload_tag(a.workload, a.f32_mode))
    roof = dict(groof, traffic=traffic, traffic_source=traffic_src, kernel=k1name,
                kernel_avg_ms=round(g["avg_ms"], 4), events_every=tstride)
    if traffic:
        roof["traffic_ratio_to_unique_bytes"] = round(traffic / (n * dl * es), 3)

    # the whole step against its floor: t_floor = max(flops_alg / fp64
    # matrix peak, bytes_alg / HBM peak) with bytes_alg = (n + m) * d_local * s + 8 d_local;
    # and K4 (k_mean, the HBM-bound kernel) against HBM: m * d_local * s + 8 d_local bytes
    bytes_alg = (n + m) * dl * es + 8 * dl
    t_mfma = (groof["ops_per_launch"] / (PEAK_I8_TOPS * 1e12) if "ops_per_launch" in groof
              else flops / (peak * 1e12)) * 1e3
    t_hbm = bytes_alg / (PEAK_HBM_GBS * 1e9) * 1e3
    step_roof = {"t_floor_ms": round(max(t_mfma, t_hbm), 4),
                 "bound": "mfma" if t_mfma >= t_hbm else "hbm",
                 "t_measured_ms": round(ms_per_step, 4),
                 "frac": round(max(t_mfma, t_hbm) / ms_per_step, 4)}
    km = kbreak.get("k_mean")
    if km:
        kb = m * dl * es + 8 * dl
        kgbs = kb / (km["avg_ms"] * 1e-3) / 1e9
        k4_roof = {"bound": "hbm", "achieved": round(kgbs, 1), "peak": PEAK_HBM_GBS,
                   "unit": "GB/s", "frac": round(kgbs / PEAK_HBM_GBS, 4), "kernel": "k_mean",
                   "kernel_avg_ms": round(km["avg_ms"], 4), "bytes_per_launch": kb}
    else:
        k4_roof = None

    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": w["dtype"],
        "data": "synthetic (repo SplitMix64 spec, generated on device; DESIGN.md)",
        "config": {"workload": a.workload, "n": n, "d": d, "f": f, "m": m,
                   "parallelism": ("d-shard x%d + %s" % (world, "host (gloo) exchange" if host_exch else
                                                         "RCCL all-gather" if a.deterministic else
                                                         "RCCL all-reduce"))
                   if sharded and not emu else
                   ("emulated rank 0 of %d (1 GPU)" % emu if emu else "1 GPU"),
                   "d_local": dl, **({"f32_mode": a.f32_mode} if w["dtype"] == "f32" or f64_i8 else {})},
        "roofline": roof,
        "roofline_hbm_k4": k4_roof,
        "step_roofline": step_roof,
        "kernels_ms_avg": {k: round(v["avg_ms"], 5) for k, v in kbreak.items()},
        "parity": parity,
    }
    if variants:
        out["variants"] = variants

    if parity is not None and not emu:
        parity["margin"] = {"near_tie": mg["near_tie"], "gap": mg["gap"],
                            "err_bound": mg["err_bound"]}

    # one verifier call after idle (the DVFS ramp), beside the steady state
    sc_step, sc_k1, sc_all = single_call(step, eng, barrier, world, dev)
    sc_gbs = n * (dl if emu else d) * es / (sc_step * 1e-3) / 1e9
    out["single_call"] = {
        "what": "median of 7 calls, each after 200 ms of GPU idle (one Multi-Krum per batch, "
                "krum.go:100-166): the clock ramp a verifier sees",
        "ms": round(sc_step, 4), "GB_per_s": round(sc_gbs, 3),
        "k_gram_ms": round(sc_k1, 4),
        "k_gram_frac": round(groof["frac"] * g["avg_ms"] / sc_k1, 4) if sc_k1 > 0 else None,
        "step_roofline_frac": round(max(t_mfma, t_hbm) / sc_step, 4),
        "calls_ms": [round(x, 4) for x in sc_all]}

    if sharded:
        # evidence that RCCL reached N ranks and that every rank selected the same set
        import hashlib
        nr, rk = eng.comm_size()
        ex, by = eng.comm_stats()
        h = hashlib.sha256(sel.cpu().numpy().tobytes()).hexdigest()[:16]
        hs = [h]
        if world > 1:
            hs = [None] * world
            tdist.all_gather_object(hs, h)
        ar = kbreak.get("allreduce")
        usz = int(_lib.lib().bk_upper_elems(n))
        comm_ranks = nr
        if host_exch:
            nr = world
        # this rank's K1 and exchange per step, from the timed region itself
        # (HIP events on libbk's stream around K1 and around the RCCL
        # all-reduce; the host exchange by the wall clock), gathered from
        # every rank
        ar_t = kt.get("allreduce")
        mine = {"rank": rank, "device": dev_idx, "d_local": dl,
                "k_gram_ms": round(g["avg_ms"], 4),
                "exchange_ms": round(host_exch_ms if host_exch else
                                     (ar_t["avg_ms"] if ar_t else float("nan")), 4)}
        per_rank = [mine]
        if world > 1:
            per_rank = [None] * world
            tdist.all_gather_object(per_rank, mine)
        ex_ms = [p["exchange_ms"] for p in per_rank]
        out["rccl"] = {
            "nranks": nr, "rank": rk,
            "mode": ("host (gloo all_reduce of the packed partials; test mode, not RCCL)"
                     if host_exch else
                     "all-gather + fixed-order sum" if a.deterministic else "all-reduce (sum)"),
            "bytes_per_exchange": usz * 8 * (nr if a.deterministic else 1),
            "comm_ranks": comm_ranks if not host_exch else None,
            "exchange_ms": round(max(ex_ms), 4),
            "exchange_ms_avg_untimed_pass": round(ar["avg_ms"], 4) if ar else None,
            "per_rank": per_rank,
            "exchanges_this_rank": ex, "bytes_this_rank": by,
            "selected_set_sha16": h, "ranks_agree": len(set(hs)) == 1}

    if rank == 0 and world == 1 and not emu and not a.no_next_rows and w["dtype"] == "f64":
        out["next_rows"] = next_rows(eng, X, n, d, sel, m)

    if rank == 0 and world == 1 and not emu and not a.no_variants and a.workload == DEFAULT_WORKLOAD:
        # the headline batch with its Gram from exact int8 digit slices, certified
        # (bk_set_f64_mode(BK_F64_I8_CERTIFIED): the selection is always the
        # reference's -- an exact re-run on a near tie -- and K4 reads the fp64
        # rows).  A variant, never `value`: the headline stays the fp64 MFMA path
        V = out.setdefault("variants", {})
        for mode in ("i8_certified", "i8x2_certified"):
            V[workload_tag(a.workload, mode)] = device_variant(eng, dev, a.workload, mode, steps=20, X=X)

    if rank == 0 and world == 1 and not emu and not a.no_variants:
        # every other single-GPU BASELINE config in the driver-timed line, each
        # with its own warm-up, roofline, hash-matched PMC traffic, parity and
        # CPU baseline at its shape
        V = out.setdefault("variants", {})
        cpu = not a.no_cpu_baseline
        if a.workload == DEFAULT_WORKLOAD:
            V["C_1024x131072"] = device_variant(eng, dev, "C_1024x131072", steps=20)
            if cpu:
                V["C_1024x131072"]["cpu_baseline"] = cpu_baseline(WORKLOADS["C_1024x131072"], 5.0, 3.0)
        if a.workload == DEFAULT_WORKLOAD or w["dtype"] == "f32":
            we = WORKLOADS["E_4096x262144_fp32"]
            XE = X if a.workload == "E_4096x262144_fp32" else None
            if XE is None:
                XE = torch.empty((we["n"], we["d"]), dtype=torch.float32, device=dev)
                eng.synth_fill_ptr(XE.data_ptr(), _lib.BK_F32, we["n"], we["d"], we["d"], 0,
                                   we["d"], we["seed"], we["nbyz"])
            for mode in ("exact", "mfma", "certified") + I8_MODE_NAMES:
                if a.workload == "E_4096x262144_fp32" and mode == a.f32_mode:
                    continue  # that is the line itself
                V[workload_tag("E_4096x262144_fp32", mode)] = device_variant(
                    eng, dev, "E_4096x262144_fp32", mode, steps=10, X=XE)
            if cpu and "E_4096x262144_fp32" in V:
                V["E_4096x262144_fp32"]["cpu_baseline"] = cpu_baseline(we, 5.0, 3.0)
            del XE
            torch.cuda.empty_cache()
        if a.workload == DEFAULT_WORKLOAD:
            for nm in ("B_mnist", "A_creditcard"):
                V[nm] = small_variant(eng, dev, nm)
                V[nm]["host_entry"] = host_entry_variant(eng, dev, nm)
                if cpu:
                    V[nm]["cpu_baseline"] = cpu_baseline(WORKLOADS[nm], 3.0, 2.0)
        if f64_i8:  # the line's own mode for what follows
            eng.set_f64_mode(F32_MODES[a.f32_mode])
        else:
            eng.set_f32_mode(F32_MODES[a.f32_mode])

    if rank == 0 and world == 1 and not emu and a.workload == DEFAULT_WORKLOAD and not a.no_graph_probe:
        out["hip_graph"] = graph_probe(eng, dev, X, n, d, f, sel, scores, mean, bdt)

    if rank == 0 and world == 1 and not emu and not a.no_e2e:
        # PCIe-inclusive rate: pinned host batch -> H2D -> Multi-Krum -> D2H of sel and mean
        import ctypes
        Xh = torch.empty((n, dl), dtype=tdt, pin_memory=True)
        Xh.copy_(X[:, :dl])
        selh = np.empty(m, dtype=np.int64)
        meanh = np.empty(dl, dtype=np.float64)
        mo = ctypes.c_int64(0)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            _lib.check(_lib.lib().bk_multikrum(eng.ctx, ctypes.c_void_p(Xh.data_ptr()),
                                               _lib.BK_HOST_PINNED, bdt, n, dl, dl, f,
                                               selh.ctypes.data, ctypes.addressof(mo), None,
                                               meanh.ctypes.data))
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        # the verifier's one call per batch after idle: the copy phase runs the
        # chunks' K1s, so the clock ramp (single_call above) is paid under it
        idle = []
        for _ in range(3):
            torch.cuda.synchronize()
            time.sleep(0.2)
            t0 = time.perf_counter()
            _lib.check(_lib.lib().bk_multikrum(eng.ctx, ctypes.c_void_p(Xh.data_ptr()),
                                               _lib.BK_HOST_PINNED, bdt, n, dl, dl, f,
                                               selh.ctypes.data, ctypes.addressof(mo), None,
                                               meanh.ctypes.data))
            idle.append((time.perf_counter() - t0) * 1e3)
        out["e2e_pinned_h2d_d2h"] = {"GB_per_s": round(n * d * es / t / 1e9, 3),
                                     "ms": round(t * 1e3, 3),
                                     "after_idle_ms": [round(x, 3) for x in idle],
                                     "selected_set_same": bool(np.array_equal(
                                         selh, sel.cpu().numpy()))}
        del Xh

    if rank == 0 and world == 1 and not emu and not a.no_e2e and w["dtype"] == "f64":
        out["e2e_noised_pinned"] = noised_probe(eng, dev, X, n, dl, f, m)

    if rank == 0 and world == 1 and not emu and not a.no_e2e and a.workload == DEFAULT_WORKLOAD:
        # the verifier's own input: n separate host rows
        out["e2e_rows"] = {}
        for nm in ("D_512x1M_f153", "B_mnist", "A_creditcard"):
            try:
                out["e2e_rows"][nm] = rows_entry_variant(eng, dev, nm)
            except Exception as e:  # noqa: BLE001 -- must not cost the headline line
                out["e2e_rows"][nm] = {"error": repr(e)}

    if rank == 0 and world == 1 and not emu and not a.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(w)
        except Exception as e:  # the oracle is optional for the GPU number itself
            out["cpu_baseline"] = {"error": repr(e)}

    if rank == 0:
        os.write(json_fd, (json.dumps(compact_line(out, a.detail_out)) + "\n").encode())
    if tdist.is_initialized():
        tdist.barrier()
        tdist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
