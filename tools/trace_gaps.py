"""Idle gaps between consecutive kernels of one training step in a rocprofv3
--kernel-trace CSV, summed by (predecessor, successor) kernel family.
  python tools/trace_gaps.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return (n[:44] + ("R3" if n.endswith("1>(g4::GroupParams)") else ""))


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "loss_kernel" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]  # one whole step: loss kernel to loss kernel
span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b]) / 1e3
agg = collections.defaultdict(list)
for i in range(a, b):
    g = int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])
    agg[(short(rows[i]["Kernel_Name"]), short(rows[i + 1]["Kernel_Name"])[:30])].append(g / 1e3)
print("step span %.1f us, kernel time %.1f us, %d kernels, gaps %.1f us"
      % (span, busy, b - a, sum(sum(v) for v in agg.values())))
for k, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 10]:
    print("%7.1f us  n=%3d avg %6.2f  %s -> %s" % (sum(v), len(v), sum(v) / len(v), k[0], k[1]))
