# kernel names / resources of hipBLASLt's picks for the step's shapes (reference point)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mm -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_torch_mm.py > $GRAFT_REPO_ROOT/gpurun_out/mm_prof.log 2>&1 || exit 1
python - <<'PY'
import csv, os
rows = list(csv.DictReader(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/prof_mm/run_kernel_trace.csv")))
seen = {}
for r in rows:
    n = r["Kernel_Name"]
    if "Cijk" not in n and "gemm" not in n.lower():
        continue
    k = (n, r["Grid_Size_X"], r["Grid_Size_Y"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    seen.setdefault(k, []).append(d)
    if len(seen[k]) == 1:
        print(n[:200], "| wg", r["Workgroup_Size_X"], "grid", r["Grid_Size_X"], r["Grid_Size_Y"], "lds", r["LDS_Block_Size"], "vgpr", r["VGPR_Count"], r["Accum_VGPR_Count"])
for k, v in seen.items():
    v.sort()
    print("%8.1f us x%d  %s grid %s %s" % (v[len(v) // 2], len(v), k[0][:90], k[1], k[2]))
PY
