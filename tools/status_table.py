"""DESIGN.md §9's status table from one bench run and the PMC records:

    python tools/status_table.py profiles/r04/bench_r4c.json profiles/r04/bench_detail_r4c.json

Prints markdown rows: per config the bench's value and ms per step, the
dominant kernel's rocprof timed-window average and the bench's frac, the PMC
traffic over the unique input bytes, the selected-set parity and the near-tie
flag."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UNIQUE = {"D_512x1M_f153": 512 * 1048576 * 8, "C_1024x131072": 1024 * 131072 * 8,
          "E_4096x262144_fp32": 4096 * 262144 * 4, "B_mnist": 100 * 7850 * 8, "A_creditcard": 10 * 25 * 8}


def pmc(tag):
    p = os.path.join(REPO, "profiles", "pmc_%s.json" % tag)
    if not os.path.exists(p):
        return None
    return json.load(open(p)).get("k_gram") or {}


def base(tag):
    for b in UNIQUE:
        if tag.startswith(b):
            return b
    return None


def row(tag, v, unit="GB/s"):
    roof = v.get("roofline") or {}
    par = v.get("parity") or {}
    if "one_launch" in v:
        par = dict(v["one_launch"].get("parity") or {}, **par)
    k = pmc(tag) or {}
    tw = k.get("timed_window_avg_ms")
    hb = k.get("hbm_bytes_per_launch")
    ub = UNIQUE.get(base(tag))
    ms = v.get("ms_per_step")
    kern = roof.get("kernel") or ""
    kname = {"k_gram": "K1i8" if "i8" in tag else "K1", "k_small": "k_small", "k_tiny": "k_tiny"}.get(kern, kern)
    if tag.startswith("A_"):
        kname = "k_tiny"
    twt = ("%.3f ms" % tw if tw >= 0.1 else "%.1f µs" % (tw * 1e3)) if tw else "-"
    mst = ("%.3f" % ms if ms >= 0.1 else "%.4f" % ms) if ms else "-"
    fr = roof.get("frac")
    tr = "%.3g GB = %.2f×" % (hb / 1e9, hb / ub) if hb and ub else "-"
    mg = (par.get("margin") or {}).get("near_tie")
    return "| %s | %s %s | %s | %s %s | %s | %s | %s | %s |" % (
        tag, v.get("value"), unit, mst, kname, twt, fr if fr is not None else "-", tr,
        par.get("selected_set", "-"), mg if mg is not None else "-")


def main():
    line = json.load(open(sys.argv[1]))
    det = json.load(open(sys.argv[2]))
    rows = [row(line["config"]["workload"], det)]
    for name, v in (det.get("variants") or {}).items():
        rows.append(row(name, v))
        he = v.get("host_entry")
        if he:
            rows.append("| %s host entry (`bk_multikrum`, pinned) | - | %.4f | H2D alone %.4f ms, over it %.4f ms | - | - | %s | - |" % (
                name, he["ms_per_call"], he["h2d_alone_ms"], he["overhead_over_h2d_ms"],
                (he.get("parity") or {}).get("selected_set")))
    print("\n".join(rows))


if __name__ == "__main__":
    main()
