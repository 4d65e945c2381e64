"""Summarise a tools/profile.sh run into profiles/: per-kernel trace stats and
PMC-derived HBM traffic per launch, corrected as MI355X_MICROARCH.md §HBM says:
FETCH_SIZE (KiB) counts HALF the bytes of wide (16 B/lane) coalesced reads --
global_load_dwordx4 and global_load_lds_dwordx4 alike -- so it is doubled for
the kernels that read that way (k_gram3, k_mean); WRITE_SIZE is exact for
16-B-per-lane stores and uncalibrated for narrower ones (noted, not scaled).

    python tools/pmc_summary.py gpurun_out/prof_<tag> <workload> <out-prefix> [warmup steps]

With warmup/steps (those of the profiled trace run: bench.py defaults, 10 and
40) the K1 row also reports the mean over the timed window of dispatches from
the per-dispatch kernel trace -- the figure bench.py's HIP events measure (the
clock ramps over the first launches, so the all-call average runs high).
"""
import collections
import csv
import json
import os
import sys

# coalesced streaming readers (128-B requests tallied at 64 B): 16 B/lane, and
# k_qsum's 8 B/lane (calibrated: doubled it equals m*d*8 exactly)
WIDE_READS = ("k_gram3", "k_mean", "k_gram<", "k_noise", "k_qsum", "k_small", "k_gram_i8", "k_i8_slice")
# the roofline kernel: K1, or the one-launch path for n <= 128 (configs A, B)
K1_NAMES = ("k_gram", "k_small", "k_tiny")


def short(name):
    s = name.replace("void ", "")
    return s.split("(")[0].replace("bk::", "")


def pass_durations(d):
    """{dispatch id: duration ms} from the PMC pass's own kernel trace
    (profile.sh runs every --pmc pass with --kernel-trace, never other domains)."""
    p = os.path.join(d, "run_kernel_trace.csv")
    out = {}
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            out[r.get("Dispatch_Id")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return out


def load_pmc(d, only=None):
    """Per kernel: mean of every counter over its dispatches, plus the physical
    shader clock per dispatch, GRBM_GUI_ACTIVE / 8 XCDs / that dispatch's own
    duration in the same pass (MI355X_MICROARCH.md, DVFS give-back).
    only(kernel, duration_ms, longest_ms_of_kernel_in_pass) -> keep the dispatch?"""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    clocks = collections.defaultdict(list)
    durs = collections.defaultdict(list)
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not sub.startswith("pmc") or not os.path.exists(p):
            continue
        dur = pass_durations(os.path.join(d, sub))
        rows = list(csv.DictReader(open(p)))
        longest = collections.defaultdict(float)
        for r in rows:
            t = dur.get(r.get("Dispatch_Id"))
            if t:
                k = short(r["Kernel_Name"])
                longest[k] = max(longest[k], t)
        seen = set()
        for r in rows:
            k = short(r["Kernel_Name"])
            t = dur.get(r.get("Dispatch_Id"))
            if only is not None and not only(k, t or 0.0, longest[k]):
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if t and (sub, r.get("Dispatch_Id")) not in seen:
                seen.add((sub, r.get("Dispatch_Id")))
                durs[k].append(t)
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and t:
                clocks[k].append(float(r["Counter_Value"]) / 8.0 / (t * 1e-3) / 1e9)
    res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
    for k, v in durs.items():
        res[k]["_dispatch_ms_mean"] = sum(v) / len(v)
        res[k]["_dispatches"] = len(v)
    for k, v in clocks.items():
        v = sorted(v)
        med = v[len(v) // 2]
        # GRBM_GUI_ACTIVE spans the pass's counter window around the dispatch:
        # for a ~20 us kernel (k_small) that window dwarfs the kernel and the
        # ratio reads above the 2.4 GHz maximum -- no clock, not a wrong one
        res[k]["_clock_ghz_median"] = med if med <= 2.45 else None
    return res


def main():
    prof, workload, out = sys.argv[1], sys.argv[2], sys.argv[3]
    stats = list(csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_stats.csv"))))
    pmc = load_pmc(prof)
    res = {}
    lines = ["# rocprofv3 summary: %s (%s)" % (workload, os.path.basename(prof)), "",
             "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    for r in stats:
        k = short(r["Name"])
        lines.append("| %s | %s | %.1f | %.2f |" % (k, r["Calls"], float(r["AverageNs"]) / 1e3,
                                                   float(r["Percentage"])))
        res.setdefault(k, {})["avg_ms_rocprof"] = float(r["AverageNs"]) / 1e6
    lines += ["", "| kernel | FETCH_SIZE KiB | read bytes (corrected) | WRITE_SIZE KiB | "
              "HBM bytes/launch | TCC hit % | MFMA busy % | eff. clock GHz |",
              "|---|---|---|---|---|---|---|---|"]
    for k, c in sorted(pmc.items()):
        if "FETCH_SIZE" not in c:
            continue
        fetch = c["FETCH_SIZE"] * 1024.0
        corr = 2.0 if any(w in k for w in WIDE_READS) else 1.0
        rd = fetch * corr
        wr = c.get("WRITE_SIZE", 0.0) * 1024.0
        hit = c.get("TCC_HIT_sum", 0.0)
        miss = c.get("TCC_MISS_sum", 0.0)
        hr = 100.0 * hit / (hit + miss) if hit + miss else float("nan")
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        # the clock from each dispatch's own duration in the PMC pass; the
        # all-call rocprof average mixes shapes (r1 reported an impossible 6.26 GHz)
        clk = c.get("_clock_ghz_median", float("nan"))
        clk = float("nan") if clk is None else clk
        simd_cycles = gui / 8.0 * 1024 if gui else 0
        mb = 100.0 * busy / simd_cycles if simd_cycles else float("nan")
        res.setdefault(k, {}).update(fetch_kib=c["FETCH_SIZE"], read_bytes_corrected=rd,
                                     write_bytes=wr, hbm_bytes_per_launch=rd + wr,
                                     tcc_hit_pct=hr, mfma_busy_pct=mb, clock_ghz=clk,
                                     fetch_correction=corr)
        lines.append("| %s | %.0f | %.3g | %.0f | %.3g | %.1f | %.1f | %.2f |" % (
            k, c["FETCH_SIZE"], rd, c.get("WRITE_SIZE", 0.0), rd + wr, hr, mb, clk))
    lines += ["", "FETCH_SIZE doubled (x2) for wide 16-B/lane reads per MI355X_MICROARCH.md §HBM;",
              "WRITE_SIZE as reported.  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)."]
    # K1 of the workload only: its dispatches within 2x of the longest k_gram
    # dispatch of each pass (bench.py also runs config B's chain, 500 launches
    # of ~20 us on the same grid, which an all-dispatch mean would average in)
    big = load_pmc(prof, only=lambda k, t, tmax: not k.startswith(K1_NAMES) or t >= 0.5 * tmax)
    k1p = next((k for k in big if k.startswith(K1_NAMES) and "FETCH_SIZE" in big[k]), None)
    if k1p:
        c = big[k1p]
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        sc = gui / 8.0 * 1024 if gui else 0
        k1corr = 2.0 if any(w in k1p for w in WIDE_READS) else 1.0  # k_tiny: narrow loads
        rd = c["FETCH_SIZE"] * 1024.0 * k1corr
        wr = c.get("WRITE_SIZE", 0.0) * 1024.0
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        pmc_k1 = dict(fetch_kib=c["FETCH_SIZE"], read_bytes_corrected=rd, write_bytes=wr,
                      hbm_bytes_per_launch=rd + wr,
                      tcc_hit_pct=100.0 * hit / (hit + miss) if hit + miss else float("nan"),
                      mfma_busy_pct=100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / sc if sc else float("nan"),
                      clock_ghz=c.get("_clock_ghz_median"), fetch_correction=k1corr,
                      pmc_dispatch_ms_mean=c.get("_dispatch_ms_mean"),
                      pmc_dispatches=c.get("_dispatches"))
        lines += ["", "K1 of the workload only (%s dispatches >= half the longest of their pass; %d over the PMC passes, "
                  "mean %.3f ms): HBM bytes/launch %.4g (read %.4g corrected, write %.4g), TCC hit %.1f%%, "
                  "MFMA busy %.1f%%, clock %s GHz" % (k1p, pmc_k1["pmc_dispatches"],
                                                      pmc_k1["pmc_dispatch_ms_mean"], rd + wr, rd, wr,
                                                      pmc_k1["tcc_hit_pct"], pmc_k1["mfma_busy_pct"],
                                                      "%.2f" % pmc_k1["clock_ghz"] if pmc_k1["clock_ghz"]
                                                      else "n/a (kernel shorter than the counter window)")]
    # the PMC passes' dominant kernel; else the first K1-family name (the
    # trace pass also holds e.g. the host-row entries' k_tiny / k_small)
    k1 = k1p if k1p in res else next((k for k in res if k.startswith(K1_NAMES)), None)
    out_json = {"workload": workload, "source": prof, "kernels": res}
    if k1:
        out_json["k_gram"] = dict(res[k1])
        if k1p:
            out_json["k_gram"].update(pmc_k1)
        tr = os.path.join(prof, "trace", "run_kernel_trace.csv")
        if len(sys.argv) > 5 and os.path.exists(tr):
            w, st = int(sys.argv[4]), int(sys.argv[5])
            # in dispatch order (the CSV's rows are not always in time order)
            rows = sorted((r for r in csv.DictReader(open(tr)) if short(r["Kernel_Name"]) == k1),
                          key=lambda r: int(r["Start_Timestamp"]))
            durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
            win = durs[w:w + st]
            if win:
                res[k1]["dispatch_ms"] = durs
                res[k1]["timed_window_avg_ms"] = sum(win) / len(win)
                out_json["k_gram"]["timed_window_avg_ms"] = sum(win) / len(win)
                lines += ["", "%s per dispatch (ms): %s" % (k1, " ".join("%.3f" % x for x in durs)),
                          "timed window (dispatches %d..%d, = bench.py's timed steps): avg %.3f ms"
                          % (w + 1, w + st, sum(win) / len(win))]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from biscotti_amd._lib import code_object_sha16
    sha = code_object_sha16(os.path.join(repo, "biscotti_amd", "libbk.so"))  # the kernels' code
    out_json["libbk_sha16"] = sha
    json.dump(out_json, open(out + ".json", "w"), indent=1)
    if k1 and "hbm_bytes_per_launch" in out_json["k_gram"]:
        # the file bench.py reads its roofline "traffic" from (only while the
        # library hash matches: bench.py checks libbk_sha16)
        pj = os.path.join(repo, "profiles", "pmc_%s.json" % workload)
        json.dump({"workload": workload, "source": "%s.json (tools/profile.sh %s)"
                   % (os.path.relpath(out, repo), os.path.basename(prof)),
                   "libbk_sha16": sha,
                   "k_gram": {k: v for k, v in out_json["k_gram"].items() if k != "dispatch_ms"}},
                  open(pj, "w"), indent=1)
    open(out + ".md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
