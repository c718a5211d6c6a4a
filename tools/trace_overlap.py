"""Overlap of kernels in a rocprofv3 kernel trace (csv): for the last STEPS
occurrences of kernel A, which kernels ran at the same time and for how long.
python tools/trace_overlap.py run_kernel_trace.csv NAME_FRAGMENT [steps]"""
import csv
import sys


def main():
    path, frag = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r["Queue_Id"]))
    rows.sort()
    hits = [r for r in rows if frag in r[2]][-steps:]
    for s, e, name, q in hits:
        print(f"{name[:60]} q{q} {(e - s) / 1e3:.1f} us")
        for s2, e2, n2, q2 in rows:
            if n2 is name or (s2, e2) == (s, e):
                continue
            ov = min(e, e2) - max(s, s2)
            if ov > 0:
                print(f"    overlaps {n2[:60]} q{q2}: {ov / 1e3:.1f} us "
                      f"(its span {(e2 - s2) / 1e3:.1f} us, start {(s2 - s) / 1e3:+.1f})")


if __name__ == "__main__":
    main()
