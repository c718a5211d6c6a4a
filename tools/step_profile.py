"""Host-side cost of one train step (collate + train_iteration, as bench.py
times it): wall ms/step vs the host's issue rate, then a cProfile of the host
Python work.
    python tools/step_profile.py [--steps 30] [--eager]"""
import argparse
import cProfile
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--eager", action="store_true")
    args = ap.parse_args()
    import bench
    trainer, data = bench.make_trainer(args.res, 0, 0, 1, True, graph=not args.eager)

    def step():
        trainer.train_iteration(data.collate([0]))

    for _ in range(12):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    for _ in range(args.steps):
        step()
        marks.append(time.perf_counter())
    t_host = marks[-1] - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    print(f"wall {t_wall / args.steps * 1e3:.3f} ms/step, host issue {t_host / args.steps * 1e3:.3f}"
          f" ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
