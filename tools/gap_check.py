"""Per-step GPU idle time (gaps between consecutive kernels) in a rocprofv3
kernel trace of bench.py, steps delimited by loss_kernel.
  python tools/gap_check.py <trace dir>"""
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "loss_kernel" in n]
for s in range(len(idx) - 1):
    a, b = idx[s], idx[s + 1]
    gaps = [int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]) for i in range(a, b)]
    span = int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])
    print("step %2d span %.2f ms, gaps > 5 us: %3d, idle %.3f ms" %
          (s, span / 1e6, sum(1 for g in gaps if g > 5000), sum(g for g in gaps if g > 0) / 1e6))
