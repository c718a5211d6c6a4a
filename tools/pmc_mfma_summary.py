"""MFMA utilisation per kernel from a rocprofv3 --pmc pass with
SQ_INSTS_VALU_MFMA_MOPS_F16/BF16 (units of 512 FLOPs) and the kernel trace
(durations): python tools/pmc_mfma_summary.py gpurun_out/pmcmfma [out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict

PEAK = 2.5e15  # dense f16 / bf16 MFMA, MI355X_MICROARCH.md
PATS = {"k_field_fwd_fused": "field_forward", "k_field_bwd": "field_backward",
        "k_render_infer": "render_infer"}


def main(d, out=None):
    vals = defaultdict(lambda: defaultdict(list))
    dur = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]].append(
                float(r["Counter_Value"]))
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[(r["Kernel_Name"], r["Dispatch_Id"])] = (int(r["End_Timestamp"]) -
                                                         int(r["Start_Timestamp"])) * 1e-9
    res = {}
    for pat, label in PATS.items():
        rows = [(k, v) for k, v in vals.items() if pat in k[0]]
        if not rows:
            continue
        tfl, secs, busy, cu = [], [], [], []
        for k, v in rows:
            mops = sum(v.get("SQ_INSTS_VALU_MFMA_MOPS_F16", [0])) + sum(
                v.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", [0]))
            t = dur.get(k)
            if not t:
                continue
            tfl.append(mops * 512.0)
            secs.append(t)
            busy.append(sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])))
            cu.append(sum(v.get("SQ_BUSY_CU_CYCLES", [0])))
        if not secs:
            continue
        f = sum(tfl) / len(tfl)
        t = sum(secs) / len(secs)
        res[label] = {"dispatches": len(secs), "mfma_flops_per_dispatch": f,
                      "avg_us": round(t * 1e6, 2), "achieved_TFLOPs": round(f / t / 1e12, 2),
                      "frac_of_peak": round(f / t / PEAK, 5),
                      "mfma_busy_over_cu_busy": round(sum(busy) / max(sum(cu), 1.0), 4)}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
