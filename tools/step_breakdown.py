"""Per-step kernel time by kernel family from a rocprofv3 kernel trace of
bench.py (timed steps only: the trace is split into steps at the Adam kernel),
plus the step's wall span and idle (no kernel running) time.
  python tools/step_breakdown.py <run_kernel_trace.csv> [n_steps]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ends = [i for i, e in enumerate(ev) if "adam_kernel" in e[2] or "adam_gcoef" in e[2]]
steps = [ev[a + 1:b + 1] for a, b in zip(ends[-n_steps - 1:-1], ends[-n_steps:])]


def family(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:70]


per = collections.defaultdict(float)
cnt = collections.defaultdict(int)
span = busy = 0.0
for st in steps:
    span += st[-1][1] - st[0][0]
    cur_s = cur_e = None
    for s, e, n in st:
        per[family(n)] += e - s
        cnt[family(n)] += 1
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
k = len(steps)
print("steps %d: wall span %.3f ms/step, kernels busy %.3f ms/step, idle %.3f ms/step"
      % (k, span / k / 1e6, busy / k / 1e6, (span - busy) / k / 1e6))
tot = sum(per.values())
for n, t in sorted(per.items(), key=lambda x: -x[1]):
    print("%-72s %5.1f/step %8.1f us avg %7.3f ms/step %5.1f%%" % (n, cnt[n] / k, t / cnt[n] / 1e3, t / k / 1e6,
                                                                   100 * t / tot))
