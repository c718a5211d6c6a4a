"""Host-side cost of the graph-replayed C2 train step: cProfile over K steps
of bench.py's loop (no sync inside), top functions by own time and by
cumulative time.  Usage: python tools/host_profile.py [K] [--module]
(--module: the eager reference-API module path, bench.py --module-path-child)"""
import cProfile
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    module = "--module" in sys.argv
    k = int(args[0]) if args else 200
    tr, data = bench.make_trainer(128, 0, 0, 1, True, graph=not module)
    if module:
        tr.native_step = False
        tr.model.fused_field = False

    def step():
        tr.train_iteration(data.collate([0]))

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"host issue {issue / k * 1e3:.3f} ms/step, wall {total / k * 1e3:.3f} ms/step")
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(k):
        step()
    prof.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
