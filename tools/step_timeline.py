"""Per-step GPU timeline of the bench step: HIP events at each step's start and
end on the launch stream (GPU busy per step, idle between steps) and the host
time of each part of train_iteration.  Diagnostic only.

    python tools/step_timeline.py [--steps 40]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--res", type=int, default=128)
    args = ap.parse_args()
    import _dfhip
    _dfhip.load()
    tr, data = bench.make_trainer(args.res, 0, 0, 1, True, graph=True)
    for _ in range(10):
        tr.train_iteration(data.collate([0]))
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    host = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        h0 = time.perf_counter()
        d = data.collate([0])
        h1 = time.perf_counter()
        ev[i][0].record()
        tr.train_iteration(d)
        ev[i][1].record()
        h2 = time.perf_counter()
        host.append((h1 - h0, h2 - h1))
    issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    busy = [a.elapsed_time(b) * 1e3 for a, b in ev]
    gaps = [ev[i][1].elapsed_time(ev[i + 1][0]) * 1e3 for i in range(args.steps - 1)]
    n = args.steps
    print(f"wall {total / n * 1e3:.3f} ms/step, host issue {issue / n * 1e3:.3f} ms/step")
    print(f"GPU per step (event span) mean {sum(busy) / n:.1f} us, min {min(busy):.1f}, "
          f"max {max(busy):.1f}")
    print(f"gap between steps mean {sum(gaps) / len(gaps):.1f} us, max {max(gaps):.1f}")
    print(f"host collate {sum(h[0] for h in host) / n * 1e6:.1f} us, train_iteration "
          f"{sum(h[1] for h in host) / n * 1e6:.1f} us")
    print("per-step GPU spans:", [round(b) for b in busy[:20]])


if __name__ == "__main__":
    main()
