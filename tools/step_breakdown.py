"""Average per-step kernel time breakdown of a rocprofv3 kernel trace of
bench.py (steps delimited by the optimizer kernel k_adam):
    python tools/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv [first_step]"""
import csv
import sys
from collections import defaultdict


def main(path, first=11):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    acc = defaultdict(float)
    walls = []
    steps = 0
    for s in range(first, len(idx) - 1):
        a, b = idx[s], idx[s + 1]
        walls.append((int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3)
        for r in rows[a + 1:b + 1]:
            name = r["Kernel_Name"]
            key = name.split("(")[0][:60] if not name.startswith("_Z") else name[:60]
            acc[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        steps += 1
    tot = sum(acc.values()) / steps
    print(f"steps {steps}: wall {sum(walls) / steps:.1f} us, kernels {tot:.1f} us")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"{v / steps:8.1f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 11)
