"""Summarise a rocprofv3 (rocpd SQLite) trace of tools/prof_noised.py: per-kernel
and per-copy-direction stats, and per bk_multikrum_noised call the H2D copy
time, the K6 time and how much of K6 ran while a copy was in flight.
usage: python tools/rocpd_noised_summary.py <results.db> > profiles/r01/<name>.md"""
import sqlite3
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def total(iv):
    return sum(b - a for a, b in iv)


def inter(x, y):
    i = j = 0
    s = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            s += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return s


db = sqlite3.connect(sys.argv[1])
ks = [(n, s, e) for n, s, e in db.execute("select name, start, end from kernels")]
cs = [(n, s, e, z) for n, s, e, z in db.execute("select name, start, end, size from memory_copies")]
agg = defaultdict(lambda: [0, 0])
for n, s, e in ks:
    short = n.split("(")[0].split("<")[0].replace("void ", "")
    agg[short][0] += 1
    agg[short][1] += e - s
print("# rocprofv3 --kernel-trace --memory-copy-trace: bk_multikrum_noised, D 512 x 2^20 fp64, k = 1\n")
print("| kernel | calls | avg ms | total ms |\n|---|---|---|---|")
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("| %s | %d | %.4f | %.3f |" % (k, c, t / c / 1e6, t / 1e6))
cagg = defaultdict(lambda: [0, 0, 0])
for n, s, e, z in cs:
    cagg[n][0] += 1
    cagg[n][1] += e - s
    cagg[n][2] += z
print("\n| copy (pinned host shows as DEVICE_TO_DEVICE) | count | total ms | GB | GB/s (busy) |\n|---|---|---|---|---|")
for k, (c, t, z) in cagg.items():
    print("| %s | %d | %.3f | %.3f | %.1f |" % (k, c, t / 1e6, z / 1e9, z / t if t else 0))
means = sorted(e for n, s, e in ks if "k_mean" in n)
print("\nPer call (window = after the previous call's k_mean):\n")
print("| call | span ms | H2D busy ms | K6 busy ms | K6 under a copy | K1..K4 ms after last copy |")
print("|---|---|---|---|---|---|")
prev = 0
for i, me in enumerate(means):
    h2d = union([(s, e) for n, s, e, z in cs if prev < s <= me])
    k6 = union([(s, e) for n, s, e in ks if prev < s <= me and "k_noise" in n])
    if not h2d:
        prev = me
        continue
    span = me - h2d[0][0]
    tail = me - h2d[-1][1]
    print("| %d | %.2f | %.2f | %.2f | %.1f%% | %.2f |" % (
        i, span / 1e6, total(h2d) / 1e6, total(k6) / 1e6,
        100.0 * inter(k6, h2d) / max(total(k6), 1), tail / 1e6))
    prev = me
