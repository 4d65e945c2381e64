"""Where the rocclr fill / copy dispatches of a run come from.

    python tools/trace_fills.py <rocprofv3 -d dir with run_kernel_trace.csv and
                                 run_hip_api_trace.csv> <out.md>

For every __amd_rocclr_fillBufferAligned / __amd_rocclr_copyBuffer dispatch:
the HIP API call that issued it (by correlation id) and whether it was
dispatched before or after the first dominant-kernel dispatch (k_gram*), and
how many fall between the first and last dominant dispatch (inside the steps).
"""
import collections
import csv
import os
import sys

BLIT = ("__amd_rocclr_fillBufferAligned", "__amd_rocclr_copyBuffer")


def main(d, out):
    kt = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    api = {}
    p = os.path.join(d, "run_hip_api_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            api[r["Correlation_Id"]] = r["Function"]
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    gram = [int(r["Start_Timestamp"]) for r in kt if "k_gram" in r["Kernel_Name"].split("(")[0]]
    first, last = (min(gram), max(gram)) if gram else (None, None)
    rows = collections.Counter()
    for r in kt:
        name = r["Kernel_Name"]
        if name not in BLIT:
            continue
        t = int(r["Start_Timestamp"])
        if first is None or t < first:
            where = "before the first k_gram"
        elif t > last:
            where = "after the last k_gram"
        else:
            where = "between k_gram dispatches (inside the steps)"
        rows[(name, api.get(r["Correlation_Id"], "?"), where)] += 1
    with open(out, "w") as f:
        f.write("# rocclr fill / copy dispatches of %s\n\n" % d)
        f.write("k_gram dispatches: %d\n\n" % len(gram))
        f.write("| dispatch | issued by (HIP API, correlation id) | when | count |\n|---|---|---|---|\n")
        for (name, fn, where), c in sorted(rows.items()):
            f.write("| %s | %s | %s | %d |\n" % (name, fn, where, c))
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
