"""GPU-side phase timeline of graph-replayed train steps (no profiler):
events recorded on the step's stream around prologue / replay / embedding
backward / optimizer; prints per-phase GPU time and host issue time.
    python tools/step_events.py [--res 128] [--steps 20]"""
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
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--cprofile", action="store_true", help="host profile of the timed steps")
    args = ap.parse_args()
    import bench
    import _dfhip
    _dfhip.load()
    trainer, data = bench.make_trainer(args.res, 0, 0, 1, True, graph=True)
    for _ in range(10):
        trainer.train_iteration(data.collate([0]))
    torch.cuda.synchronize()
    g = next(iter(trainer._graphs.values()))
    ev = []
    marks = {}
    orig_replay, orig_load, orig_opt = g.replay, g.load, trainer.optimizer_step

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append((name, e, time.perf_counter()))

    def load(*a, **k):
        mark("load")
        return orig_load(*a, **k)

    def replay():
        mark("replay")
        g.graph.replay()
        mark("emb_bwd")
        if g.native is not None:
            g.native.embedding_backward()
        for launch, _ in g.deferred:
            launch()
        for p, gr in g.grads:
            p.grad = gr

    def opt_step():
        mark("optim")
        orig_opt()
        mark("end")

    g.load, g.replay, trainer.optimizer_step = load, replay, opt_step
    prof = None
    if args.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.train_iteration(data.collate([0]))
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof).sort_stats("tottime").print_stats(25)
    tot = {}
    htot = {}
    for (n0, e0, h0), (n1, e1, h1) in zip(ev, ev[1:]):
        if n0 == "end":
            n0 = "between"
        tot[n0] = tot.get(n0, 0.0) + e0.elapsed_time(e1)
        htot[n0] = htot.get(n0, 0.0) + (h1 - h0) * 1e3
    print(f"wall {wall / args.steps * 1e3:.3f} ms/step, host issue {host / args.steps * 1e3:.3f}")
    for k in tot:
        print(f"  {k:10s} gpu {tot[k] / args.steps:.3f} ms   host {htot[k] / args.steps:.3f} ms")


if __name__ == "__main__":
    main()
