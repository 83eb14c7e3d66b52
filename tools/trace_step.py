"""Per-step breakdown from a rocprofv3 kernel trace: kernel time by (name, grid),
and idle gaps between consecutive dispatches (launch/dependency bubbles).
usage: python tools/trace_step.py run_kernel_trace.csv [first_adam_index]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(adam) // 2
lo, hi = adam[k - 1] + 1, adam[k] + 1   # one step: after one Adam through the next
step = rows[lo:hi]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = 0
gaps = []
last_end = None
agg = defaultdict(lambda: [0, 0.0])
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if last_end is not None:
        gaps.append(max(0, s - last_end))
    last_end = max(e, last_end or 0)
    busy += e - s
    name = r["Kernel_Name"]
    for pre in ("void (anonymous namespace)::", "(anonymous namespace)::", "_ZN12_GLOBAL__N_1"):
        if name.startswith(pre):
            name = name[len(pre):]
    key = (name[:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[key][0] += 1
    agg[key][1] += (e - s) / 1e3
print("dispatches %d  wall %.3f ms  kernel-sum %.3f ms  gaps %.3f ms (n>2us: %d)" % (
    len(step), (t1 - t0) / 1e6, busy / 1e6, sum(gaps) / 1e6, sum(g > 2000 for g in gaps)))
for key, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%8.1f us  %3d x %8.1f  %-60s grid %s,%s,%s" % (us, n, us / n, key[0], key[1], key[2], key[3]))
