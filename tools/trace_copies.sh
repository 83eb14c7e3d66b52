# kernel sequence of one bench step, to see where the D2D copies (copyBuffer) sit
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/trace_copy -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-traffic --steps 1 --warmup 1 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/trace_copy.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, os
f = glob.glob(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/trace_copy/**/*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"][:60] for r in rows]
# the last step: from the last loss_kernel back to the previous loss_kernel
idx = [i for i, n in enumerate(names) if "loss_kernel" in n]
a = idx[-2] + 1 if len(idx) > 1 else 0
b = len(names)
for i in range(a, b):
    if "copyBuffer" in names[i] or "Fill" in names[i] or "elementwise" in names[i]:
        d = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
        print(i - a, "%.1fus" % d, names[i], "| prev:", names[i - 1], "| next:", names[i + 1] if i + 1 < b else "")
PY
