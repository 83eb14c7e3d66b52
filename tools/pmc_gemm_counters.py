"""Per-kernel mean of SQ counters over the GEMM (or other: 2nd argument, a name
substring) dispatches of a rocprofv3 --pmc run.
  python tools/pmc_gemm_counters.py <dir> [name-filter]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "gemm"
vals = defaultdict(lambda: defaultdict(dict))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if flt not in n:
            continue
        k = int(r["Dispatch_Id"])
        c = r["Counter_Name"]
        vals[n][c][k] = vals[n][c].get(k, 0.0) + float(r["Counter_Value"])
for n, cs in sorted(vals.items()):
    short = n.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0][:60]
    parts = []
    for c, dk in sorted(cs.items()):
        parts.append("%s=%.3g" % (c, sum(dk.values()) / len(dk)))
    print("%-60s n=%d %s" % (short, len(next(iter(cs.values()))), " ".join(parts)))
