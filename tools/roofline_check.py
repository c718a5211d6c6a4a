"""Reproduce bench.py's roofline line from a rocprofv3 kernel trace of the
same child command bench.py profiles (tools/gpu_round.sh):

    python tools/roofline_check.py BENCH_JSON KERNEL_TRACE_CSV [keep] [--shading]

--shading: the line's shading.roofline (the textureless step's grid embedding
backward) against a trace of `bench.py --shade textureless` (the same child).

Region time = the last `keep` dispatches of each of the region's kernels
(bench.REGION_KERNELS), averaged; bytes = the line's bytes_per_launch (the
region's byte model at the child's samples per step).  Prints the recomputed
achieved GB/s and frac next to the line's, and their ratio."""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main(bench_json, trace_csv, keep=16, shading=False):
    import bench
    d = json.loads([l for l in open(bench_json) if l.startswith("{")][-1])
    roof = d["shading"]["roofline"] if shading else d["roofline"]
    region = roof.get("region", roof["kernel"])
    pats = bench.REGION_KERNELS.get(region, (region,))
    durs = {}
    for r in csv.DictReader(open(trace_csv)):
        for i, alts in enumerate(pats):
            alts = (alts,) if isinstance(alts, str) else alts
            if any(a in r["Kernel_Name"] for a in alts):
                durs.setdefault(i, []).append((int(r["Start_Timestamp"]),
                                               int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    us = sum(sum(v for _, v in sorted(x)[-keep:]) / keep / 1e3 for x in durs.values())
    gbs = roof["bytes_per_launch"] / (us * 1e-6) / 1e9
    frac = gbs / roof["peak"]
    print(json.dumps({"region": region, "shading": shading, "trace_us": round(us, 2),
                      "line_us": roof["avg_us"], "trace_GBs": round(gbs, 1),
                      "line_GBs": roof["achieved"], "trace_frac": round(frac, 4),
                      "line_frac": roof["frac"], "ratio": round(frac / roof["frac"], 3)}))


if __name__ == "__main__":
    flags = [a for a in sys.argv[1:] if a.startswith("--")]
    pos = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(pos[0], pos[1], int(pos[2]) if len(pos) > 2 else 16, shading="--shading" in flags)
