"""CPU-side cost of one train step: wall time per step, and the torch.profiler
table of host ops (where the launch/sync gaps come from).
    python tools/step_profile.py [--steps 10]"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--res", type=int, default=128)
    args = ap.parse_args()
    import bench
    trainer, data = bench.make_trainer(args.res, 0, 0, 1, True)
    batches = [data.collate([i]) for i in range(16)]
    for i in range(10):
        trainer.train_iteration(batches[i % 16])
    torch.cuda.synchronize()
    # wall vs host time
    t0 = time.perf_counter()
    for i in range(args.steps):
        trainer.train_iteration(batches[i % 16])
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    print(f"wall {t_wall / args.steps * 1e3:.3f} ms/step, host returns after "
          f"{t_host / args.steps * 1e3:.3f} ms/step")
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for i in range(args.steps):
            trainer.train_iteration(batches[i % 16])
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=45))


if __name__ == "__main__":
    main()
