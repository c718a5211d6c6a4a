"""Benchmark: SDS train steps/s and rays/s at 128x128 on 1..8 MI355X.

One step = one iteration of the reference's training loop (nerf/utils.py:
693-715) with the -O preset (fp16 autocast, cuda_ray, dir_text): random orbit
camera -> 128x128 rays -> occupancy-grid march -> tiled-grid encoder ->
MLP -> compositing -> SDS gradient (synthetic stand-in, no SD weights exist
offline) + entropy regulariser -> backward -> GradScaler/Adam step, with the
density-grid refresh every 16 steps.  Multi-GPU: one process per GPU, each
rank renders its own seed (data parallel over views), gradients all-reduced
over RCCL before the optimizer step (weak scaling).

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "single-stable-dreamfusion_amd"
for _p in (str(ROOT), str(PKG)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "SDS train steps/sec + rays/sec at 128×128, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ATOMIC_PEAK_GBS = 1300.0     # MI355X_MICROARCH.md: global float atomics ~1.3 TB/s


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--res", type=int, default=128)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--two-pass-backward", action="store_true",
                   help="reference double backward instead of the fused single pass")
    p.add_argument("--mock-sds", action="store_true",
                   help="SyntheticSDS (SDS arithmetic around stand-in VAE/UNet) instead of the "
                        "injected w(t) N(0,1) gradient")
    p.add_argument("--eager", action="store_true",
                   help="launch every kernel eagerly (no HIP-graph replay of the step)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--cpu-steps", type=int, default=1)
    return p.parse_args()


def make_trainer(res, seed, rank, world, fused, graph=False, mock_sds=False):
    import main
    from nerf.network_grid import NeRFNetwork
    from nerf.provider import NeRFDataset
    from nerf.sd import InjectedSDS, SyntheticSDS
    from nerf.utils import Trainer, make_adam, seed_everything

    opt = main.parse_opt(["--text", "a hamburger", "-O", "--h", str(res), "--w", str(res),
                          "--guidance", "synthetic", "--seed", str(seed)])
    # identical model initialisation on every rank; per-rank RNG (cameras,
    # march noise, background, SDS draws) from here on
    seed_everything(seed)
    device = torch.device("cuda", torch.cuda.current_device())
    model = NeRFNetwork(opt)
    seed_everything(seed + rank)
    guidance = SyntheticSDS(device) if mock_sds else InjectedSDS(device)
    optimizer = lambda m: make_adam(m.get_params(opt.lr), betas=(0.9, 0.99), eps=1e-15)  # noqa
    sched = lambda o: torch.optim.lr_scheduler.LambdaLR(o, lambda it: 0.1 ** min(it / opt.iters, 1))  # noqa
    trainer = Trainer("df", opt, model, guidance, device=device, workspace=None,
                      optimizer=optimizer, ema_decay=None, fp16=True, lr_scheduler=sched,
                      use_checkpoint="scratch", scheduler_update_every_step=True,
                      local_rank=rank, world_size=world, mute=True, fused_backward=fused,
                      graph_step=graph)
    data = NeRFDataset(opt, device=device, type="train", H=res, W=res, size=100)
    trainer.model.train()
    return trainer, data


def cpu_baseline(res, steps):
    """The oracle's pure-PyTorch CPU restatement of the --cuda_ray-off train
    step, on this host's cores, over a bounded sample."""
    import oracle.cpu_render as cr
    cores = len(os.sched_getaffinity(0))
    threads = int(os.environ.get("OMP_NUM_THREADS", cores))
    torch.set_num_threads(max(1, min(cores, threads)))
    step = cr.CPUTrainStep(res, res, seed=0)
    step.step()  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        step.step()
    dt = time.perf_counter() - t0
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": res * res * steps / dt, "unit": "rays/s", "steps_per_sec": steps / dt,
            "cores": torch.get_num_threads(), "kind": "port", "cpu_model": model,
            "sample": f"{steps} timed + 1 warm-up --cuda_ray-off train steps at {res}x{res} "
                      f"(64 coarse + 64 importance samples/ray, fp32, synthetic SDS, Adam)"}


def summarize_kernels(records):
    torch.cuda.synchronize()
    per = {}
    import _dfhip
    for name, e0, e1, nbytes in records:
        ms = e0.elapsed_time(e1)
        d = per.setdefault(name, [0.0, 0, 0])
        d[0] += ms
        d[1] += 1
        d[2] += _dfhip.record_bytes(nbytes)
    out = {}
    for name, (ms, n, nbytes) in per.items():
        avg_ms = ms / n
        gbs = (nbytes / n) / (avg_ms * 1e-3) / 1e9
        out[name] = {"launches": n, "avg_us": round(avg_ms * 1e3, 2), "total_ms": round(ms, 3),
                     "bytes_per_launch": int(nbytes / n), "achieved_GBs": round(gbs, 1)}
    return out


# timed region -> its kernels, each as alternative name fragments (rocprofv3
# reports some names demangled, some mangled)
REGION_KERNELS = {
    "grid_encode_backward": (("gb::k_bin", "gb5k_bin"), ("gb::k_walk", "gb6k_walk"),
                             ("gb::k_sum", "gb5k_sum")),
    "grid_field_forward": ("k_field_fwd_fused",),
    "field_mlp_backward": ("k_field_bwd", "k_field_wgrad_sum"),
    "grid_encode_forward": ("k_grid_fwd",),
    "march_rays_train_count": ("k_march_train_count",),
    "march_rays_train_emit": ("k_march_train_emit",),
    "composite_rays_train_forward": ("k_composite_train_fwd",),
    "composite_rays_train_backward": ("k_composite_train_bwd",),
}


def load_pmc(name):
    """Per-launch HBM bytes of timed region `name` (sum over its kernels) from
    the committed rocprofv3 PMC summary (profiles/pmc_summary.json, made by
    tools/gpu_pmc_bench.sh + tools/pmc_summary.py), or None."""
    path = ROOT / "profiles" / "pmc_summary.json"
    if not path.exists():
        return None
    try:
        data = json.loads(path.read_text())
    except ValueError:
        return None
    kernels = data.get("kernels", {})
    total = 0
    for pats in REGION_KERNELS.get(name, (name,)):
        pats = (pats,) if isinstance(pats, str) else pats
        hit = next((v for k, v in kernels.items() if any(p in k for p in pats)), None)
        if hit is None:
            return None  # a kernel of the region was not profiled
        total += hit["hbm_bytes_per_dispatch"]
    return total


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)

    import _dfhip
    _dfhip.load()
    trainer, data = make_trainer(args.res, args.seed, rank, world, not args.two_pass_backward,
                                 graph=not (args.eager or args.two_pass_backward),
                                 mock_sds=args.mock_sds)

    def step():
        trainer.train_iteration(data.collate([0]))

    for _ in range(args.warmup):
        step()

    timer = None
    if not args.no_kernel_timing:
        timer = _dfhip.new_kernel_timer()
        _dfhip.set_kernel_timer(timer)
    counts = []

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        counts.append(trainer.model.step_counter[(trainer.model.local_step - 1) % 16, 0].clone())
    host_issue = time.perf_counter() - t0  # host done issuing (no sync inside the loop)
    barrier()
    elapsed = time.perf_counter() - t0
    _dfhip.set_kernel_timer(None)

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    samples = float(torch.stack(counts).float().mean().item())
    kernels = summarize_kernels(timer.records) if timer else {}

    rays_per_step = args.res * args.res
    steps_per_sec = args.steps * world / elapsed  # whole-job aggregate (every rank steps)
    value = rays_per_step * args.steps * world / elapsed
    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "rays/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp16+f32",
        "data": "synthetic: random orbit cameras, random-init grid network, "
                + ("SDS arithmetic around stand-in VAE/UNet" if args.mock_sds else
                   "seeded w(t)*N(0,1) SDS gradient injected at pred_rgb")
                + " (no SD-1.5 weights offline)",
        "config": {"workload": f"C2: -O (fp16, cuda_ray, dir_text) {args.res}x{args.res} render, "
                               f"batch 1, max_steps 512, density grid update every 16 steps",
                   "global_batch": world, "rays_per_step_per_gpu": rays_per_step,
                   "parallelism": f"dp{world}",
                   "backward": "two-pass (reference)" if args.two_pass_backward else "fused",
                   "launch": "eager" if not trainer.graph_step else "hip-graph replay",
                   "mean_samples_per_step": round(samples, 1)},
        "steps_per_sec": round(steps_per_sec, 3),
        "host_issue_ms_per_step": round(host_issue / args.steps * 1e3, 3),
    }
    if kernels:
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        kd = kernels[dom]
        traffic = load_pmc(dom)
        result["roofline"] = {
            "kernel": dom, "bound": "hbm", "achieved": kd["achieved_GBs"], "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(kd["achieved_GBs"] / HBM_PEAK_GBS, 4),
            "traffic": traffic, "avg_us": kd["avg_us"],
            "bytes_per_launch": kd["bytes_per_launch"]}
        result["kernels"] = kernels
        step_ms = result["ms_per_step"]
        result["kernel_share_of_step"] = {k: round(v["total_ms"] / args.steps / step_ms, 4)
                                          for k, v in kernels.items()}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.res, args.cpu_steps)
        result["gpu_vs_cpu"] = round(value / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
