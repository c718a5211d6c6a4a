"""Top kernels of a rocprofv3 --stats kernel_stats.csv:
    python tools/prof_top.py gpurun_out/prof/run_kernel_stats.csv [N]"""
import csv
import sys


def main(path, n=20):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
        print(f"{r['Name'][:80]:80s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f}us "
              f"{100 * float(r['TotalDurationNs']) / tot:5.1f}%")
    print(f"total {tot / 1e6:.2f} ms, {sum(int(r['Calls']) for r in rows)} launches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
