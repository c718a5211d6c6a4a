"""Per-workgroup walk timeline (tools/walk_trace.py's report) of the C2 bench
step itself: the bench trainer (graph-replayed native step) warms up, then
one eager-twin step runs with the walk trace installed.
python tools/walk_trace_bench.py [--warmup 20] [--steps 3]"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tools")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--shade", default="albedo", help="albedo | textureless | lambertian")
    args = ap.parse_args()
    import _dfhip
    import bench
    from gridencoder.grid import level_offsets
    from walk_trace import report
    import _gridencoder
    _dfhip.load()
    trainer, data = bench.make_trainer(args.res, 0, 0, 1, True, graph=True)
    if args.shade != "albedo":
        trainer.pick_shading = (lambda k: (lambda: (k, 0.1)))(args.shade)

    def step():
        trainer.train_iteration(data.collate([0]))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    trace = torch.zeros(8 * 8192, dtype=torch.int64, device="cuda")
    pls = np.exp2(np.log2(2048 / 16) / 15)
    offs = level_offsets(16, 2, 3, 16, pls, 16, False).astype(np.int32)
    trainer.step_hook = lambda g: g.step_timed()
    g = next(iter(trainer._graphs.values()))
    # the eager twin's embedding backward with a walk trace (per-call options)
    g.native.binned_opts = _gridencoder.BinnedOpts(trace=trace)
    g.native._emb_launch = None
    for i in range(args.steps):
        trace.zero_()
        torch.cuda.synchronize()
        step()
        torch.cuda.synchronize()
        ns = getattr(g, "native", None) or getattr(g, "step", None)
        M = int(ns.m_dev.item()) if ns is not None and hasattr(ns, "m_dev") else 1
        print(f"--- step {i} (samples {M})")
        report(trace, M, 16, offs, shift=13)
    trainer.step_hook = None


if __name__ == "__main__":
    main()
