"""Summarise tools/profile_roni.sh (SURVEY §8(f) row 4's kernels) into
profiles/: each kernel's dispatch time, and what binds it, from counters:

  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
  VALU busy  = 4 SQ_ACTIVE_INST_VALU   / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
  LDS busy   = 4 SQ_ACTIVE_INST_LDS    / (GRBM_GUI_ACTIVE / 8 x 256 CUs)
  HBM        = (2 FETCH_SIZE + WRITE_SIZE) KiB / dispatch time / 8 TB/s
  waiting    = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on memory / barriers)
  occupancy  = SQ_WAVE_CYCLES / 4 / (GRBM_GUI_ACTIVE / 8) / 256 CUs (resident waves per CU)
(quad-cycle counters x 4; GRBM_GUI_ACTIVE is summed over the 8 XCDs --
MI355X_MICROARCH.md, PMC units).  The binding resource is the busiest of
MFMA / VALU / LDS / HBM; a kernel whose waves mostly wait, at low occupancy
and with every busy fraction low, is latency-bound: its floor is the launch
(an empty dispatch's duration, from the same trace) plus its critical path.

    python tools/roni_pmc_summary.py gpurun_out/prof_roni profiles/r06/pmc_roni_r06
"""
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary as P  # noqa: E402

KERNELS = {  # libbk call -> its dispatches
    "K7 bk_roni (logistic)": ("k_roni_mm_prep<false>", "k_roni_sign_reg<1>", "k_roni_sign_reg<2>", "k_roni_sign", "k_roni_score"),
    "K8 bk_roni_softmax (one batch)": ("k_roni_xnorm", "k_roni_mm_prep<true>", "k_roni_wnorm",
                                       "k_roni_logits", "k_roni_mc_score"),
    "K8 bk_roni_softmax_batches": ("k_roni_batch",),
}


def trace_durations(prof):
    rows = list(csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_trace.csv"))))
    d = {}
    for r in rows:
        d.setdefault(P.short(r["Kernel_Name"]), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return d


def main():
    prof, out = sys.argv[1], sys.argv[2]
    pmc = P.load_pmc(prof)
    durs = trace_durations(prof)
    # the empty-dispatch floor: the shortest 1-workgroup torch kernel of the trace
    tiny = [min(v) for k, v in durs.items() if "elementwise_kernel" in k]
    floor_us = min(tiny) if tiny else None
    res = {"launch_floor_us": floor_us, "kernels": {}}
    lines = ["# rocprofv3 record: SURVEY §8(f) row 4 kernels (%s)" % os.path.basename(prof), "",
             "| kernel | us (median) | MFMA busy | VALU busy | LDS busy | HBM frac | waiting | waves/CU | binds |",
             "|---|---|---|---|---|---|---|---|---|"]
    for call, ks in KERNELS.items():
        for k in ks:
            c = pmc.get(k, {})
            us = statistics.median(durs[k]) if k in durs else None
            g = c.get("GRBM_GUI_ACTIVE")
            cyc = g / 8.0 if g else None

            def frac(num, units, scale=1.0):
                return (scale * c[num] / (cyc * units)) if cyc and num in c else None
            mf = frac("SQ_VALU_MFMA_BUSY_CYCLES", 1024)
            va = frac("SQ_ACTIVE_INST_VALU", 1024, 4.0)
            ld = frac("SQ_ACTIVE_INST_LDS", 256, 4.0)
            hbm = None
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c and us:
                hbm = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0 / (us * 1e-6) / 8e12
            wait = (c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]) if c.get("SQ_WAVE_CYCLES") else None
            occ = (c["SQ_WAVE_CYCLES"] / cyc / 256.0) if cyc and "SQ_WAVE_CYCLES" in c else None
            busy = {"mfma": mf, "valu": va, "lds": ld, "hbm": hbm}
            top = max(((v, n) for n, v in busy.items() if v is not None), default=(None, None))
            binds = top[1]
            if top[0] is not None and top[0] < 0.3 and wait is not None and wait > 0.5:
                binds = "latency (%s %.2f busiest; waves parked %.0f%%)" % (top[1], top[0], 100 * wait)
            res["kernels"][k] = {"call": call, "us_median": us, "mfma_busy": mf, "valu_busy": va,
                                 "lds_busy": ld, "hbm_frac": hbm, "wait_frac": wait,
                                 "waves_per_cu": occ, "binds": binds,
                                 "clock_ghz": c.get("_clock_ghz_median"),
                                 "counters": {n: v for n, v in c.items() if not n.startswith("_")}}
            f = lambda x: "-" if x is None else "%.3f" % x  # noqa: E731
            lines.append("| %s | %s | %s | %s | %s | %s | %s | %s | %s |" % (
                k, f(us), f(mf), f(va), f(ld), f(hbm), f(wait), f(occ), binds))
    lines += ["", "Launch floor (the shortest 1-workgroup dispatch in the same trace): %s us" %
              ("-" if floor_us is None else "%.2f" % floor_us)]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from biscotti_amd._lib import code_object_sha16
    res["libbk_sha16"] = code_object_sha16(os.path.join(repo, "biscotti_amd", "libbk.so"))  # the kernels' code
    res["source"] = "%s.json (tools/profile_roni.sh)" % os.path.relpath(out, repo)
    with open(out + ".json", "w") as fp:
        json.dump(res, fp, indent=1)
    # the file bench.py's next_rows reads (only while the library hash matches)
    with open(os.path.join(repo, "profiles", "pmc_roni.json"), "w") as fp:
        json.dump(res, fp, indent=1)
    with open(out + ".md", "w") as fp:
        fp.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
