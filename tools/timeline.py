"""One train step's kernel timeline from a rocprofv3 kernel trace (the step
between two consecutive launches of a marker kernel):
    python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [marker] [min_us]"""
import csv
import sys


def main(path, marker="k_walk", min_us=0.0):
    t = list(csv.DictReader(open(path)))
    t.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(t) if marker in r["Kernel_Name"]]
    a, b = idx[-3], idx[-2]
    seg = t[a + 1:b + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print(f"kernels {len(seg)}  span {(t1 - t0) / 1e3:.1f} us  busy {busy / 1e3:.1f} us")
    prev = None
    small, small_n = 0.0, 0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        prev = e
        d = (e - s) / 1e3
        if d >= min_us or gap >= 5:
            print(f"{(s - t0) / 1e3:8.1f} {d:7.1f} gap{gap:6.1f}  {r['Kernel_Name'][:90]}")
        else:
            small += d
            small_n += 1
    print(f"({small_n} kernels under {min_us} us: {small:.1f} us)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_walk",
         float(sys.argv[3]) if len(sys.argv) > 3 else 0.0)
