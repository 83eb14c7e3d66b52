"""Per-launch GEMM times of the C5 step, bf16 vs fp8 (tools/run_c5_trace.sh):
the GEMM launches of the last traced step of each run, aligned by their order
in the step (the launch sequence is the same; fp8 adds only quantization
kernels), grouped by (bf16 kernel, fp8 kernel) pair.
  python tools/c5_gemm_compare.py <trace dir bf16> <trace dir fp8>"""
import csv
import glob
import sys
from collections import defaultdict


def gemm_launches(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # steps end at the optimizer's Adam launch: keep the last complete step
    ends = [i for i, n in enumerate(names) if "adam" in n]
    lo, hi = ends[-2] + 1, ends[-1] + 1
    out = []
    for r in rows[lo:hi]:
        n = r["Kernel_Name"]
        if "gemm" in n.lower() and "quant" not in n.lower():
            short = n.replace("(anonymous namespace)::", "").split("(")[0]
            out.append((short, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out


a, b = gemm_launches(sys.argv[1]), gemm_launches(sys.argv[2])
print("GEMM launches per step: bf16 %d, fp8 %d" % (len(a), len(b)))
if len(a) != len(b):
    sys.exit("launch sequences differ")
grp = defaultdict(list)
for (na, ta), (nb, tb) in zip(a, b):
    if na != nb:
        grp[(na, nb)].append((ta, tb))
for (na, nb), v in sorted(grp.items(), key=lambda kv: -len(kv[1])):
    ta = sum(x for x, _ in v) / len(v)
    tb = sum(y for _, y in v) / len(v)
    print("%3d x  bf16 %-55s %7.1f us   fp8 %-40s %7.1f us  (%+.1f us)" % (len(v), na[:55], ta, nb[:40], tb, tb - ta))
    # per-launch detail: launches in step order
    print("      per launch (bf16 / fp8 us): " + ", ".join("%.0f/%.0f" % p for p in v[:16]))
tot_a = sum(t for _, t in a)
tot_b = sum(t for _, t in b)
print("GEMM time per step: bf16 %.2f ms, fp8 %.2f ms" % (tot_a / 1e3, tot_b / 1e3))
