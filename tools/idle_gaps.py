"""Idle time between kernels in a rocprofv3 kernel trace of bench.py: per timed
step, the step's wall span (first kernel start to last kernel end) vs the sum
of kernel durations (merged intervals, so overlapping kernels count once).
  python tools/idle_gaps.py <run_kernel_trace.csv> [n_steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# steps end with adam_kernel: split on them
ends = [i for i, e in enumerate(ev) if "adam_kernel" in e[2] or "adam_gcoef" in e[2]]
steps = []
prev = None
for i in ends[-n_steps:]:
    j = prev + 1 if prev is not None else None
    prev = i
    if j is not None:
        steps.append(ev[j:i + 1])
tot_span = tot_busy = 0
gaps = []
for st in steps:
    span = st[-1][1] - st[0][0]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in st:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot_span += span
    tot_busy += busy
print("steps %d: span %.3f ms/step, kernels busy %.3f ms/step, idle %.3f ms/step (%.1f%%), %d gaps/step, median gap %.2f us"
      % (len(steps), tot_span / len(steps) / 1e6, tot_busy / len(steps) / 1e6, (tot_span - tot_busy) / len(steps) / 1e6,
         100.0 * (tot_span - tot_busy) / tot_span, len(gaps) // max(1, len(steps)), sorted(gaps)[len(gaps) // 2] / 1e3))
