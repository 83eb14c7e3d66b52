"""Effective clock of each kernel family under load (MI355X_MICROARCH.md, 'DVFS
give-back'): GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / kernel wall time,
from one rocprofv3 run with --pmc GRBM_GUI_ACTIVE and --kernel-trace.

  python tools/pmc_clock.py <dir> <out.json> <tag>"""
import csv
import glob
import json
import os
import sys


def family(name):
    for key, fam in (("gemm256r_group", "gemm_grouped_dW"), ("gemm256f8", "gemm_fp8"), ("gemm256r", "gemm_ring"),
                     ("gemm_kernel", "gemm_128"), ("attn_bwd", "attn_bwd"), ("attn_fwd", "attn_fwd"),
                     ("ln_bwd", "ln_bwd"), ("ln_fwd", "ln_fwd"), ("adam", "adam")):
        if key in name:
            return fam
    return None


def main():
    d, out, tag = sys.argv[1:4]
    active = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                k = int(r["Dispatch_Id"])
                active[k] = active.get(k, 0.0) + float(r["Counter_Value"])
    dur, names = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            names[k] = r["Kernel_Name"]
    fams = {}
    for k, a in active.items():
        if k not in dur or dur[k] < 3e-4:  # the quotient reads high below ~0.3 ms (guide)
            continue
        fam = family(names[k])
        if fam is None:
            continue
        s = fams.setdefault(fam, [0.0, 0.0, 0])
        s[0] += a / 8.0
        s[1] += dur[k]
        s[2] += 1
    res = {"tag": tag, "method": "rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace; clock = sum(GRBM_GUI_ACTIVE/8) / sum(wall) "
                                 "over dispatches >= 0.3 ms of the profiled bench run (profiled runs clock ~2-5 % low)",
           "families": {f: {"dispatches": n, "ghz": round(c / t / 1e9, 3)} for f, (c, t, n) in fams.items()}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
