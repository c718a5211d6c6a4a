"""Summarise rocprofv3 counter CSVs (p*_counter_collection.csv) per kernel:
mean counter value per dispatch.  python tools/pmc_table.py gpurun_out/pmcg"""
import csv
import glob
import sys
from collections import defaultdict


def main(d, pat=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        if pat and pat not in k:
            continue
        if not pat and "grid" not in k and "sum_partials" not in k:
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcg",
         sys.argv[2] if len(sys.argv) > 2 else None)
