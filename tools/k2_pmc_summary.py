"""Per-kernel PMC averages from rocprofv3 --pmc passes (counter_collection csv):
    python tools/k2_pmc_summary.py <dir> [kernel substring]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "k_scores2"
vals = defaultdict(list)
for path in sorted(glob.glob(root + "/**/*counter_collection.csv", recursive=True)):
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if want in r.get("Kernel_Name", ""):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print("%-28s n=%3d  mean %.4g" % (k, len(v), sum(v) / len(v)))
