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
    p.add_argument("--cpu-steps", type=int, default=3)
    p.add_argument("--c1-steps", type=int, default=10,
                   help="timed CPU iterations of BASELINE configs[0] (64x64), 0 to skip")
    p.add_argument("--no-infer", action="store_true",
                   help="skip the C4 inference-render measurement")
    p.add_argument("--infer-res", type=int, default=800)
    p.add_argument("--no-shading", action="store_true",
                   help="skip timing the textureless / lambertian steps")
    p.add_argument("--no-alt-backward", action="store_true",
                   help="skip timing the other backward structure (two-pass / fused)")
    p.add_argument("--no-module-path", action="store_true",
                   help="skip timing the reference-module path (autograd through the "
                        "reference-API encoder / MLP modules, no fused field, no native step)")
    p.add_argument("--module-path-child", action="store_true",
                   help="(internal) run the step through the reference-API modules: the "
                        "Trainer's autograd body, GridEncoder -> MLP -> trunc_exp / sigmoid "
                        "-> composite_rays_train as separate nodes")
    p.add_argument("--no-c5", action="store_true",
                   help="skip the C5 leg (256x256 bf16 renderer step)")
    p.add_argument("--c5-res", type=int, default=256)
    p.add_argument("--no-traffic", action="store_true",
                   help="skip the live rocprofv3 PMC passes for roofline.traffic")
    p.add_argument("--shade", default="albedo", choices=("albedo", "textureless", "lambertian"),
                   help="shading of the timed steps (the shading roofline's profiled child "
                        "runs the textureless step; the headline is albedo)")
    p.add_argument("--launcher-selftest", action="store_true",
                   help="CPU/gloo check of the N-rank launch only (no GPU work)")
    return p.parse_args()


def env_options(model=None, trainer=None):
    """A/B switches of tools/ scripts, read from the environment here only (the
    package itself takes them as explicit options): DFHIP_NATIVE_STEP,
    DFHIP_NATIVE_ADAM, DFHIP_KEPT_CLEAN, DFHIP_COMBINED_HEAD, DFHIP_STENCIL_BIN
    (Trainer), DFHIP_FUSED_FIELD,
    DFHIP_INFER_QUADS, DFHIP_INFER_ORDER, DFHIP_INFER_CHUNK_LOG2, DFHIP_INFER_TILES=0,
    DFHIP_INFER_OVERLAP_BG=0 (renderer),
    DFHIP_GRID_BWD=atomic (GridEncoder)."""
    env = os.environ
    if trainer is not None:
        for name, attr in (("DFHIP_NATIVE_STEP", "native_step"),
                           ("DFHIP_NATIVE_ADAM", "native_optimizer"),
                           ("DFHIP_KEPT_CLEAN", "kept_clean_scratch"),
                           ("DFHIP_COMBINED_HEAD", "combined_head"),
                           ("DFHIP_STENCIL_BIN", "stencil_bin")):
            if name in env:
                setattr(trainer, attr, env[name] != "0")
        model = trainer.model if model is None else model
    if model is not None:
        if "DFHIP_FUSED_FIELD" in env:
            model.fused_field = env["DFHIP_FUSED_FIELD"] != "0"
        if "DFHIP_INFER_QUADS" in env:
            model.infer_quads = env["DFHIP_INFER_QUADS"] != "0"
        if "DFHIP_INFER_ORDER" in env:
            model.infer_order = int(env["DFHIP_INFER_ORDER"])
        if "DFHIP_INFER_CHUNK_LOG2" in env:
            model.infer_chunk_log2 = int(env["DFHIP_INFER_CHUNK_LOG2"])
        if env.get("DFHIP_INFER_TILES") == "0":  # 64-ray row strips as queue chunks
            model.infer_tile_w = 0
        if env.get("DFHIP_INFER_OVERLAP_BG") == "0":  # background net after the render
            model.infer_overlap_bg = False

        enc = getattr(model, "encoder", None)
        if env.get("DFHIP_GRID_BWD") == "atomic" and hasattr(enc, "backward_mode"):
            enc.backward_mode = "atomic"


def make_trainer(res, seed, rank, world, fused, graph=False, mock_sds=False, bf16=False):
    """bf16: BASELINE configs[4] (C5) — bf16 autocast, SD-2.1-base text width."""
    import main
    from nerf.network_grid import NeRFNetwork
    from nerf.provider import NeRFDataset
    from nerf.sd import InjectedSDS, SyntheticSDS
    from nerf.utils import Trainer, make_adam, seed_everything

    opt = main.parse_opt(["--text", "a hamburger", "-O", "--h", str(res), "--w", str(res),
                          "--guidance", "synthetic", "--seed", str(seed)]
                         + (["--bf16", "--sd_version", "2.1-base"] if bf16 else []))
    # identical model initialisation on every rank; per-rank RNG (cameras,
    # march noise, background, SDS draws) from here on
    seed_everything(seed)
    device = torch.device("cuda", torch.cuda.current_device())
    model = NeRFNetwork(opt)
    seed_everything(seed + rank)
    text_dim = 1024 if bf16 else 768
    guidance = (SyntheticSDS(device, text_dim=text_dim) if mock_sds
                else InjectedSDS(device, text_dim=text_dim))
    optimizer = lambda m: make_adam(m.get_params(opt.lr), betas=(0.9, 0.99), eps=1e-15)  # noqa
    sched = lambda o: torch.optim.lr_scheduler.LambdaLR(o, lambda it: 0.1 ** min(it / opt.iters, 1))  # noqa
    trainer = Trainer("df", opt, model, guidance, device=device, workspace=None,
                      optimizer=optimizer, ema_decay=None, fp16=not bf16, bf16=bf16,
                      lr_scheduler=sched,
                      use_checkpoint="scratch", scheduler_update_every_step=True,
                      local_rank=rank, world_size=world, mute=True, fused_backward=fused,
                      graph_step=graph)
    data = NeRFDataset(opt, device=device, type="train", H=res, W=res, size=100)
    trainer.model.train()
    env_options(trainer=trainer)
    return trainer, data


def replica_digest(trainer):
    """f64 digest of one rank's replica state (every parameter, the Adam step
    counts and moments, the GradScaler scale, the density grid and bitfield):
    per tensor its sum and its sum of squares.  Data-parallel ranks that stay
    replicas (the reference's DDP contract, nerf/utils.py:200-202) have equal
    digests bit for bit."""
    m = trainer.model
    ts = [p.detach() for p in m.parameters()]
    for st in trainer.optimizer.state.values():
        for k in ("step", "exp_avg", "exp_avg_sq"):
            if k in st and torch.is_tensor(st[k]):
                ts.append(st[k])
    if trainer.scaler.is_enabled():
        ts.append(torch.as_tensor(trainer.scaler.get_scale(), dtype=torch.float64))
    if getattr(m, "cuda_ray", False):
        ts += [m.density_grid, m.density_bitfield]
    dev = next(m.parameters()).device
    out = []
    for t in ts:
        t = t.to(device=dev, dtype=torch.float64)
        out += [t.sum(), (t * t).sum()]
    return torch.stack(out)


def replica_check(trainer, samples, world):
    """After the timed region: replicas_identical (MIN == MAX of every digest
    entry over the ranks) and every rank's mean samples per step."""
    d = replica_digest(trainer)
    lo, hi = d.clone(), d.clone()
    per_rank = [samples]
    if world > 1:
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        s = torch.tensor([samples], dtype=torch.float64, device=d.device)
        got = [torch.zeros_like(s) for _ in range(world)]
        dist.all_gather(got, s)
        per_rank = [float(g.item()) for g in got]
    return bool(torch.equal(lo, hi)), [round(v, 1) for v in per_rank]


def cpu_baseline(res, steps, c1_steps=10, c1_warmup=3):
    """The oracle's pure-PyTorch CPU restatement of the --cuda_ray-off train
    step (renderer.py:301-443 run() + sample_pdf, grid network, entropy, Adam)
    on this host's cores, with the GPU leg's guidance (w(t) N(0,1) injected at
    pred_rgb): `steps` timed steps (+1 warm-up) at the GPU workload's res x res
    (the reported value), and BASELINE configs[0] = C1, 64x64 with c1_steps
    timed iterations after c1_warmup warm-up ones."""
    import oracle.cpu_render as cr
    cores = len(os.sched_getaffinity(0))
    threads = int(os.environ.get("OMP_NUM_THREADS", cores))
    torch.set_num_threads(max(1, min(cores, threads)))

    def timed(r, k, w):
        step = cr.CPUTrainStep(r, r, seed=0, guidance="injected")
        for _ in range(w):
            step.step()
        t0 = time.perf_counter()
        for _ in range(k):
            step.step()
        return (time.perf_counter() - t0) / k

    dt = timed(res, steps, 1)
    c1 = timed(64, c1_steps, c1_warmup) if c1_steps > 0 else None
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    out = {"value": res * res / dt, "unit": "rays/s", "steps_per_sec": 1.0 / dt,
           "cores": torch.get_num_threads(), "kind": "port", "cpu_model": model,
           "sample": f"{steps} timed + 1 warm-up --cuda_ray-off train steps at {res}x{res} "
                     f"(64 coarse + 64 importance samples/ray, fp32, w(t) N(0,1) SDS gradient "
                     f"injected at pred_rgb as on the GPU, entropy, Adam)"}
    if c1 is not None:
        out["c1"] = {"workload": "C1: main.py -O off, 64x64, run() 64+64 samples, fp32, CPU",
                     "steps": c1_steps, "warmup": c1_warmup, "ms_per_step": round(c1 * 1e3, 1),
                     "steps_per_sec": round(1.0 / c1, 4), "rays_per_sec": round(4096 / c1, 1)}
    return out


def sphere_occupancy_(model, radius=0.5):
    """SURVEY §8d preset R1: the analytic sphere |x| < radius written straight
    into the occupancy state (density grid 1 inside, 0 outside; bitfield by
    packbits at 0.5), for a sample count that does not depend on the field."""
    import raymarching
    xyzs, indices = model._grid_points()
    inside = (xyzs.norm(dim=-1) < radius).float()
    with torch.no_grad():
        model.density_grid[0, indices.long()] = inside
        raymarching.packbits(model.density_grid, 0.5, model.density_bitfield)


def bench_inference(device, res=800, frames=10, warmup=3, loop_frames=2, seed=1,
                    occupancy="grid"):
    """C4 (BASELINE configs[3]): res x res inference render of run_cuda's eval
    branch (albedo, fp16 autocast, max_steps 512, T_thresh 1e-4) from the
    reference's test-view camera.  occupancy "grid": the occupancy comes from
    update_extra_state of a seeded network with U(-0.5, 0.5) embeddings
    (SURVEY §8d preset R0; no trained checkpoint exists offline); "sphere":
    the analytic radius-0.5 sphere (preset R1) with the same field.  Times
    the fused persistent renderer (the product path) and, for comparison, the
    reference-structured host loop (march_rays -> field -> composite_rays with
    one sync per iteration, renderer.py:496-532) on the same kernels."""
    import main
    import _dfhip
    from nerf.network_grid import NeRFNetwork
    from nerf.provider import NeRFDataset
    opt = main.parse_opt(["--text", "a hamburger", "-O", "--h", str(res), "--w", str(res)])
    torch.manual_seed(seed)
    model = NeRFNetwork(opt).to(device)
    model.infer_tile_w = res  # the frame's rays are one res x res image: 8 x 8 tile chunks
    env_options(model=model)
    with torch.no_grad():
        model.encoder.embeddings.uniform_(-0.5, 0.5)
    with torch.autocast("cuda", dtype=torch.float16):
        for _ in range(3):
            model.update_extra_state()
    if occupancy == "sphere":
        sphere_occupancy_(model)
    model.eval()
    data = NeRFDataset(opt, device=device, type="test", H=res, W=res, size=8).collate([1])
    rays_o, rays_d = data["rays_o"], data["rays_d"]
    n = rays_o.shape[0] * rays_o.shape[1]

    def frame():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            return model.render(rays_o, rays_d, staged=True, perturb=False, light_d=None,
                                ambient_ratio=1.0, shading="albedo", force_all_rays=True,
                                bg_color=None, **vars(opt))

    def timed_frames(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            frame()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k

    model.native_infer = True
    for _ in range(warmup):
        frame()
    timer = _dfhip.new_kernel_timer()
    _dfhip.set_kernel_timer(timer)
    fused_s = timed_frames(frames)
    _dfhip.set_kernel_timer(None)
    kall = summarize_kernels(timer.records)
    kern = kall.get("render_rays_infer", {})
    korder = kall.get("render_ray_order", {})
    work = model.last_infer_work.cpu().numpy().view(np.uint32)
    samples = int(work[1]) + (int(work[2]) << 32)
    occ = ("occupancy from update_extra_state of a seeded U(-0.5,0.5) grid network (R0)"
           if occupancy == "grid" else "analytic radius-0.5 sphere occupancy (R1), same field")
    out = {"workload": f"C4: {res}x{res} run_cuda eval render (albedo, fp16, max_steps 512, "
                       f"T_thresh 1e-4), test-view camera, {occ}",
           "rays_per_frame": n, "ms_per_frame": round(fused_s * 1e3, 3),
           "rays_per_sec": round(n / fused_s, 1), "samples_per_frame": samples,
           "launch": "queue order (k_chunk_cost + k_chunk_order: render_ray_order, "
                     "order_avg_us) then ONE persistent kernel (k_render_infer, kernel_avg_us) "
                     "with the background net (k_head_fwd_net) on a side stream beside it, "
                     "then the mix (k_head_fwd_plain)"}
    if korder:
        out["order_avg_us"] = korder["avg_us"]
    if kern:
        t = kern["avg_us"] * 1e-6
        flops = 12800.0 * samples  # sigma MLP forward, SURVEY §8d
        out["kernel_avg_us"] = kern["avg_us"]
        out["samples_per_sec"] = round(samples / t, 1)
        out["mfma"] = {"achieved": round(flops / t / 1e12, 2), "peak": 2500.0,
                       "unit": "TFLOP/s", "frac": round(flops / t / 2.5e15, 5)}
        # what the reference's loop moves through HBM for the same work
        # (SURVEY §8d C4 line: 212 B per sample + 96 B per ray)
        out["unfused_equivalent_GBs"] = round((212.0 * samples + 96.0 * n) / t / 1e9, 1)
    if loop_frames > 0:
        model.native_infer = False
        frame()
        loop_s = timed_frames(loop_frames)
        model.native_infer = True
        out["loop_ms_per_frame"] = round(loop_s * 1e3, 3)
        out["speedup_vs_loop"] = round(loop_s / fused_s, 2)
    return out


def bench_c5(args, rank, world):
    """BASELINE configs[4] (C5), renderer leg: the same train step at
    c5_res x c5_res (65,536 rays) under bf16 autocast — bf16 table, features,
    activations and colours (csrc/fieldmlp.hip bf16 instantiations on
    v_mfma_f32_16x16x32_bf16), no GradScaler — graph-replayed, with the
    injected w(t) N(0,1) guidance of SD-2.1-base's text width (1024); the
    SD-2.1-base UNet / VAE cannot be loaded offline, so the full SDS step is
    not timed."""
    tr, dat = make_trainer(args.c5_res, args.seed, rank, world, True, graph=not args.eager,
                           mock_sds=args.mock_sds, bf16=True)
    for _ in range(args.warmup):
        tr.train_iteration(dat.collate([0]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_iteration(dat.collate([0]))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    last = min(16, args.steps)
    rows = [(tr.model.local_step - 1 - i) % 16 for i in range(last)]
    samples = float(tr.model.step_counter[rows, 0].float().mean().item())
    n = args.c5_res * args.c5_res
    g = next(iter(tr._graphs.values()), None)
    out = {"workload": f"C5 renderer leg: {args.c5_res}x{args.c5_res} render, bf16 autocast "
                       "(bf16 field on v_mfma_f32_16x16x32_bf16, no GradScaler), cuda_ray, "
                       "max_steps 512, injected w(t)*N(0,1) guidance (SD-2.1-base weights "
                       "not available offline)",
           "dtype": "bf16+f32", "rays_per_step": n, "steps": args.steps,
           "ms_per_step": round(dt * 1e3, 3), "steps_per_sec": round(1.0 / dt, 3),
           "rays_per_sec": round(n / dt, 1), "mean_samples_per_step": round(samples, 1),
           "native_step": bool(g is not None and g.native is not None)}
    if not args.no_kernel_timing:
        kern, info = kernel_timing_pass(tr, lambda: tr.train_iteration(dat.collate([0])), 5)
        out["kernels"], out["kernel_timing"] = kern, info
    fm = field_mlp_report(tr)
    if fm:
        out["field_mlp"] = fm
    del tr, dat
    torch.cuda.empty_cache()
    return out


MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16 / bf16 MFMA


def field_mlp_report(trainer):
    """MFMA throughput of the fused field kernels of the train step (the
    sigma MLP): the last step's fused forward (grid gather
    + 32-64-64-4 MLP) and MLP backward re-launched eagerly and timed with
    events.  Algorithmic FLOPs per field row: forward 2 x (32x64 + 64x64 +
    64x4) = 12,800; backward 2 x that for the input and weight
    gradients = 25,600 (the kernel's recompute of the forward is not
    counted)."""
    g = next(iter(trainer._graphs.values()), None) if getattr(trainer, "_graphs", None) else None
    nat = getattr(g, "native", None)
    if nat is None:
        return None
    fwd_us, bwd_us, rows = nat.time_field()
    out = {"rows": rows}
    for name, us, per in (("forward", fwd_us, 12800.0), ("backward", bwd_us, 25600.0)):
        tf = per * rows / (us * 1e-6) / 1e12
        out[name] = {"avg_us": round(us, 2), "flops_per_row": per,
                     "mfma": {"achieved": round(tf, 2), "peak": MFMA_PEAK_TFLOPS,
                              "unit": "TFLOP/s", "frac": round(tf / MFMA_PEAK_TFLOPS, 5)}}
    return out


SPIN_CYCLES = 4_000_000  # > the eager step's host issue time (~1 ms)


def kernel_timing_pass(trainer, step, k):
    """Per-kernel HIP-event timings of the train step, measured right after the
    timed region in the same process: k more steps in which every graphed
    native step runs its eager twin (GraphedTrainStep.step_timed: the same
    launches, arguments and buffers the replay runs) with a kernel timer
    installed, so each launch is bracketed by events on its launch stream.
    The timed region itself replays graphs with no events inside; the
    rocprofv3 kernel trace of a bench run (profiles/) times the replayed
    kernels for comparison.  Returns (summary per region, info)."""
    import _dfhip
    eager = not trainer.graph_step
    trainer.step_hook = None if eager else (lambda g: g.step_timed())
    timer = _dfhip.new_kernel_timer()
    _dfhip.set_kernel_timer(timer)
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            # a spin kernel holds the stream while the host issues the whole
            # eager step, so its launches then run back to back as in the graph
            # and no region's events bracket host launch gaps
            torch.cuda._sleep(SPIN_CYCLES)
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / k
    finally:
        _dfhip.set_kernel_timer(None)
        trainer.step_hook = None
    info = {"steps": k, "ms_per_step_incl_spin": round(dt * 1e3, 3), "models": dict(timer.models),
            "note": (f"HIP events around each launch on its stream, {k} steps of the eager twin "
                     "of the replayed native step run after the timed region"
                     if not eager else f"HIP events around each launch, {k} eager steps")}
    return summarize_kernels(timer.records), info


# SURVEY §8(d) per-step algorithmic byte model of the reference's op sequence
# (each logical operand once, backward once): 472 M + 492 N + 50.85 MB
def survey_step_bytes(M, N):
    return 472.0 * M + 492.0 * N + 28.0 * 1_816_247


def step_roofline(kernels, steps, M, N, trainer):
    """SURVEY §8(d) step-level roofline: sum of every timed region's
    algorithmic bytes / sum of their kernel time, per step, against the HBM
    peak; with each region's bytes per launch, time and share."""
    tot_b = sum(v["bytes_per_launch"] * v["launches"] for v in kernels.values()) / steps
    tot_us = sum(v["total_ms"] for v in kernels.values()) * 1e3 / steps
    gbs = tot_b / (tot_us * 1e-6) / 1e9
    per = {k: {"bytes_per_launch": v["bytes_per_launch"], "avg_us": v["avg_us"],
               "launches_per_step": round(v["launches"] / steps, 3),
               "achieved_GBs": v["achieved_GBs"],
               "frac": round(v["achieved_GBs"] / HBM_PEAK_GBS, 4),
               "share_of_kernel_time": round(v["total_ms"] * 1e3 / steps / tot_us, 4)}
           for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["total_ms"])}
    sb = survey_step_bytes(M, N)
    return {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "bytes_per_step": int(tot_b), "kernel_us_per_step": round(tot_us, 2),
            "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "frac_of_measured_6290": round(gbs / 6290.0, 4),
            "survey_model_bytes_per_step": int(sb),
            "survey_model_GBs": round(sb / (tot_us * 1e-6) / 1e9, 1),
            "note": "bytes: each region's compulsory operand bytes at this path's dtypes "
                    "(nerf/native_step.py timed regions); survey_model: SURVEY 8(d) "
                    "472 M + 492 N + 50.85 MB over the same kernel time",
            "kernels": per}


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
    "grid_encode_backward": (("gb::k_bin", "gb5k_bin"),
                             ("gb::k_walk", "gb6k_walk", "gb11k_walk_flat"),
                             ("gb::k_sum", "gb5k_sum")),
    "grid_field_forward": ("k_field_fwd_fused",),
    "field_mlp_backward": ("k_field_bwd", "k_field_wgrad_sum"),
    "grid_encode_forward": ("k_grid_fwd",),
    "march_rays_train_count": ("k_march_train_count",),
    "march_rays_train_emit": ("k_march_train_emit",),
    "composite_rays_train_forward": ("k_composite_train_fwd",),
    "composite_rays_train_backward": ("k_composite_train_bwd",),
}


MEASURE_TRAFFIC_DETAIL = {}  # region -> per-kernel bytes of the last measure_traffic
MEASURE_TRAFFIC_CHILD_M = {}  # region -> the profiled child's mean samples per step
MEASURE_TRAFFIC_TRACE_US = {}  # region -> its kernels' replayed duration per step (child trace)
MEASURE_STEP_TRACE_US = {}  # "step" -> every kernel's replayed duration per step (child trace)


def measure_traffic(region, timeout=180, warmup=10, shade="albedo", key=None):
    """HBM bytes per launch of timed region `region`, measured now: rocprofv3
    passes over a short child run of this same bench (graph-replayed steps, no
    extras), each its own run as MI355X_MICROARCH.md prescribes: a plain
    kernel trace (the replayed kernels' durations: MEASURE_TRAFFIC_TRACE_US),
    --pmc FETCH_SIZE, --pmc WRITE_SIZE, --pmc TCC_HIT_sum + TCC_MISS_sum.
    FETCH_SIZE is doubled (the gfx950 correction for wide reads; the guide
    leaves gathers uncalibrated), both are KiB.  The child's samples per step
    are recorded so bytes, time and traffic are compared at ONE workload.
    shade: the child's step shading (the shaded step's roofline profiles the
    textureless step); key: the name its figures are recorded under
    (default: region).  Returns (bytes or None, note)."""
    key = key or region
    import shutil
    import signal
    import subprocess
    import tempfile
    import csv
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not on PATH"
    # the child runs as many steps as this process's warm-up + timed region
    # (the occupancy grid, and with it M, grows over the first hundred
    # steps): its last `keep` steps, the ones profiled, sit where the timed
    # region ends
    # profiled steps: 16, so the window holds exactly one density refresh (one
    # step in 16, as in the timed region) and averages the random cameras'
    # samples per step (they vary 3x)
    keep = 16
    child = [sys.executable, str(Path(__file__).resolve()), "--steps", str(keep), "--warmup",
             str(max(1, warmup)),
             "--no-cpu-baseline", "--no-kernel-timing", "--no-alt-backward", "--no-shading",
             "--no-infer", "--no-traffic", "--no-c5", "--no-module-path", "--shade", shade]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    env["TMPDIR"] = "/tmp"
    tmp = tempfile.mkdtemp(prefix="dfhip_pmc_", dir="/tmp")
    pats = REGION_KERNELS.get(region, (region,))
    per = {}
    # FETCH_SIZE and WRITE_SIZE each in a run of its own; then the L2 hit /
    # miss split (TCC_HIT / TCC_MISS, 2 TCC counters), which says how much of
    # the fetch the region's requests caused versus re-read from L2
    child_m = []
    trace_us = None
    for counters in ((), ("FETCH_SIZE",), ("WRITE_SIZE",), ("TCC_HIT_sum", "TCC_MISS_sum")):
        tag = counters[0] if counters else "TRACE"
        d = os.path.join(tmp, tag)
        if counters:
            cmd = [rp, "--kernel-trace", "--pmc", *counters, "--output-format", "csv", "-d", d,
                   "-o", "run", "--"] + child
        else:  # the replayed graph's kernel durations (no counters)
            cmd = [rp, "--kernel-trace", "--stats", "--output-format", "csv", "-d", d,
                   "-o", "run", "--"] + child
        with open(os.path.join(tmp, tag + ".out"), "w") as out:
            proc = subprocess.Popen(cmd, stdout=out, stderr=subprocess.DEVNULL, env=env,
                                    start_new_session=True)
            try:
                rc = proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()
                return None, f"{tag} pass timed out"
        if rc != 0:
            return None, f"{tag} pass exited {rc}"
        try:  # the child's samples per step (the traffic scales with it)
            line = [l for l in open(os.path.join(tmp, tag + ".out")) if l.startswith("{")][-1]
            child_m.append(json.loads(line)["config"]["mean_samples_per_step"])
        except (IndexError, ValueError, KeyError):
            pass
        if not counters:
            durs = {}
            for f in Path(d).rglob("*kernel_trace.csv"):
                for r in csv.DictReader(open(f)):
                    for i, alts in enumerate(pats):
                        alts = (alts,) if isinstance(alts, str) else alts
                        if any(a in r["Kernel_Name"] for a in alts):
                            durs.setdefault(i, []).append(
                                (int(r["Start_Timestamp"]),
                                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
            if len(durs) != len(pats):
                return None, "kernel trace: not every kernel of the region was traced"
            # the last `keep` dispatches of each kernel (one per step)
            trace_us = {i: sum(v for _, v in sorted(x)[-keep:]) / keep / 1e3
                        for i, x in durs.items()}
            # every kernel of the last `keep` steps (from the keep-th last step
            # prologue on): the replayed step's kernel time
            allk = []
            for f in Path(d).rglob("*kernel_trace.csv"):
                for r in csv.DictReader(open(f)):
                    allk.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                 r["Kernel_Name"]))
            starts = sorted(t0 for t0, _, n in allk if "k_step_prologue" in n)
            if len(starts) >= keep and key == region:
                b0 = starts[-keep]
                MEASURE_STEP_TRACE_US["step"] = sum(
                    t1 - t0 for t0, t1, _ in allk if t0 >= b0) / keep / 1e3
            continue
        sums = {}
        for f in Path(d).rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                name = r.get("Counter_Name", tag)
                for i, alts in enumerate(pats):
                    alts = (alts,) if isinstance(alts, str) else alts
                    if any(a in r["Kernel_Name"] for a in alts):
                        did = int(r.get("Dispatch_Id", 0) or 0)
                        sums.setdefault((i, name), []).append((did, float(r["Counter_Value"])))
        for cname in counters:
            got = {i: [v for _, v in sorted(vs)[-keep:]] for (i, n), vs in sums.items()
                   if n == cname}
            if len(got) != len(pats):
                return None, f"{cname}: not every kernel of {region} was profiled"
            scale = {"FETCH_SIZE": 2.0 * 1024.0, "WRITE_SIZE": 1024.0}.get(cname, 1.0)
            per[cname] = {i: scale * sum(v) / len(v) for i, v in got.items()}
    shutil.rmtree(tmp, ignore_errors=True)
    total = sum(per["FETCH_SIZE"].values()) + sum(per["WRITE_SIZE"].values())
    names = [a if isinstance(a, str) else a[0] for a in pats]
    MEASURE_TRAFFIC_CHILD_M[key] = (sum(child_m) / len(child_m)) if child_m else None
    MEASURE_TRAFFIC_DETAIL[key] = {
        names[i]: {"fetch_x2": int(per["FETCH_SIZE"][i]), "write": int(per["WRITE_SIZE"][i]),
                   "l2_hit_rate": round(per["TCC_HIT_sum"][i] /
                                        max(1.0, per["TCC_HIT_sum"][i] + per["TCC_MISS_sum"][i]),
                                        4),
                   "replayed_us": round(trace_us[i], 2)}
        for i in range(len(pats))}
    MEASURE_TRAFFIC_TRACE_US[key] = sum(trace_us.values())
    return int(total), (
        "measured in this run: rocprofv3 --pmc passes (separate runs: FETCH_SIZE, WRITE_SIZE, "
        "TCC_HIT_sum + TCC_MISS_sum) of a child bench ending where the timed region ends, the "
        "last 16 dispatches of each kernel; FETCH_SIZE x2 (the gfx950 correction, calibrated for 16-B streaming loads "
        "only: an upper bound for gathers; it also counts Infinity-Cache hits), KiB -> bytes, "
        "summed over the region's kernels, mean per launch; l2_hit_rate per kernel")


MODULE_GROUPS = (  # rocprofv3 kernel name fragment -> breakdown group
    ("k_march_train", "march_rays_train"), ("k_grid_fwd", "grid_encode_forward"),
    ("k_mlp_fwd", "mlp_forward"), ("k_field_bwd", "mlp_backward"),
    ("k_field_wgrad_sum", "mlp_backward"), ("k_blc_to_lbc", "grid_encode_backward"),
    ("gb::k_", "grid_encode_backward"), ("gb5k_", "grid_encode_backward"),
    ("gb6k_", "grid_encode_backward"), ("gb11k_", "grid_encode_backward"),
    ("k_composite_train", "composite_rays_train"), ("hd::k_", "ray_head_and_entropy"),
    ("hd4k_", "ray_head_and_entropy"), ("k_entropy", "ray_head_and_entropy"),
    ("opt::k_", "adam"), ("opt5k_", "adam"), ("k_get_rays", "camera_and_near_far"),
    ("k_near_far", "camera_and_near_far"), ("occ::k_", "occupancy_refresh"),
    ("k_grid_ema", "occupancy_refresh"), ("k_packbits", "occupancy_refresh"),
    ("k_mean_count", "occupancy_refresh"), ("Cijk_", "hipblaslt_gemm"),
    ("at::native", "torch_elementwise_and_reductions"), ("rocclr", "runtime_copies_and_fills"))


def _module_breakdown(csv_files, steps):
    """Kernel time per step by group over `steps` whole steps of the child —
    from the march count launch `steps + 1` launches before its last one up
    to that last one (a step starts at its march count launch), so neither
    the child's final step nor its post-run checks are counted — from
    rocprofv3 kernel traces."""
    import csv
    ks = []
    for f in csv_files:
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    starts = [t0 for t0, _, n in ks if "k_march_train_count" in n]
    if len(starts) < steps + 1:
        return None
    b0, b1 = starts[-steps - 1], starts[-1]
    groups, top = {}, {}
    for t0, t1, n in ks:
        if t0 < b0 or t0 >= b1:
            continue
        g = next((grp for frag, grp in MODULE_GROUPS if frag in n), "other")
        groups[g] = groups.get(g, 0.0) + (t1 - t0) / 1e3 / steps
        short = n.split("(")[0][:60]
        top[short] = top.get(short, 0.0) + (t1 - t0) / 1e3 / steps
    tot = sum(groups.values())
    return {"kernel_us_per_step": round(tot, 1),
            "groups_us_per_step": {k: round(v, 1) for k, v in
                                   sorted(groups.items(), key=lambda kv: -kv[1])},
            "top_kernels_us_per_step": {k: round(v, 1) for k, v in
                                        sorted(top.items(), key=lambda kv: -kv[1])[:12]}}


def module_path_leg(args, timeout=300):
    """The C2 step through the reference-API modules one by one — GridEncoder,
    the sigma_net MLP, trunc_exp / sigmoid, composite_rays_train and the ray
    head as separate autograd nodes, the Trainer's autograd backward — with
    the reference's host-count march (`step_counter[0].item()`,
    raymarching.py:224) and the rest of the step replayed from a graph per
    sample-count bucket (nerf/graph.py BucketedModuleStep).  The path the
    reference's nerf/network_grid.py takes on this package.  A child bench
    times it, a second child the same modules launched eagerly op by op
    (`eager_ms_per_step`, the reference's launch structure exactly), and a
    third runs under rocprofv3 --kernel-trace for the per-kernel breakdown of
    the graph-replayed child's last steps."""
    import shutil
    import subprocess
    import tempfile
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    env["TMPDIR"] = "/tmp"
    cmd = [sys.executable, str(Path(__file__).resolve()), "--steps", str(min(args.steps, 20)),
           "--warmup", str(args.warmup), "--module-path-child", "--no-cpu-baseline",
           "--no-kernel-timing", "--no-alt-backward", "--no-shading", "--no-infer",
           "--no-traffic", "--no-c5", "--no-module-path"]
    try:
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
    except (subprocess.TimeoutExpired, IndexError, ValueError) as e:
        return {"error": f"{type(e).__name__}"}
    res = {"ms_per_step": d["ms_per_step"], "value": d["value"], "unit": d["unit"],
           "mean_samples_per_step": d["config"]["mean_samples_per_step"],
           "launch": "host-count march (the reference's raymarching.py:224 sync) run eagerly, "
                     "then the rest of the step (field modules -> compositing -> head -> loss "
                     "-> autograd backward) replayed from a HIP graph captured per sample-count "
                     "bucket (<= 1.25 x the count; nerf/graph.py BucketedModuleStep)",
           "note": "reference-API modules as separate autograd nodes: GridEncoder (binned "
                   "embedding backward), sigma_net MLP (dfhip_mlp_forward / _backward), "
                   "trunc_exp / gaussian / sigmoid in torch, composite_rays_train, ray head"}
    try:
        out = subprocess.run(cmd + ["--eager"], env=env, capture_output=True, text=True,
                             timeout=timeout)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
        res["eager_ms_per_step"] = json.loads(line)["ms_per_step"]
    except (subprocess.TimeoutExpired, IndexError, ValueError) as e:
        res["eager_ms_per_step"] = f"error: {type(e).__name__}"
    rp = shutil.which("rocprofv3")
    if rp is None or args.no_traffic:
        return res
    tmp = tempfile.mkdtemp(prefix="dfhip_module_", dir="/tmp")
    try:
        pcmd = [rp, "--kernel-trace", "--output-format", "csv", "-d", tmp, "-o", "run", "--",
                *cmd]
        r = subprocess.run(pcmd, env=env, capture_output=True, text=True, timeout=timeout)
        if r.returncode == 0:
            bd = _module_breakdown(list(Path(tmp).rglob("*kernel_trace.csv")), 16)
            if bd:
                res["breakdown"] = dict(bd, source="rocprofv3 --kernel-trace of the same child "
                                        "command, 16 whole steps before its last (one density "
                                        "refresh)")
    except subprocess.TimeoutExpired:
        res["breakdown_error"] = "rocprofv3 pass timed out"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return res


def shading_roofline(trainer, args):
    """The textureless step's dominant kernel region, the grid embedding
    backward over 7-point stencil groups (k_bin_fast<7> + k_walk_flat<7> +
    k_sum2), on ONE workload: a child bench replaying textureless steps
    (--shade textureless), its last 16 steps profiled by rocprofv3 (kernel
    trace, FETCH_SIZE, WRITE_SIZE, TCC hit / miss; measure_traffic).  Bytes
    per launch: SURVEY 8(d)'s model per group (its position 12 B + the seven
    rows' feature gradients 7 L C 2 B) at the child's groups per step, plus
    the table gradient once (4 rows C)."""
    m = trainer.model
    enc = m.encoder
    L, C = int(enc.num_levels), int(enc.level_dim)
    rows = int(enc.offsets_host[-1])
    traffic, note = measure_traffic("grid_encode_backward", warmup=max(1, args.warmup + args.steps - 16),
                                    shade="textureless", key="shaded_grid_encode_backward")
    cm = MEASURE_TRAFFIC_CHILD_M.get("shaded_grid_encode_backward")
    tus = MEASURE_TRAFFIC_TRACE_US.get("shaded_grid_encode_backward")
    if not (cm and tus):
        return {"kernel": "grid_encode_backward (stencil groups)", "traffic": traffic,
                "traffic_source": note}
    per = 12 + 7 * L * C * 2
    cb = 4 * rows * C + per * cm
    gbs = cb / (tus * 1e-6) / 1e9
    return {
        "kernel": "grid_encode_backward (stencil groups: k_bin_fast<7> + k_walk_flat<7> + k_sum2)",
        "region": "grid_encode_backward", "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": note,
        "traffic_by_kernel": MEASURE_TRAFFIC_DETAIL.get("shaded_grid_encode_backward"),
        "avg_us": round(tus, 2), "bytes_per_launch": int(cb), "groups_per_step": round(cm, 1),
        "algorithmic_bytes_per_group": round(cb / cm, 2),
        "traffic_per_group": round(traffic / cm, 2) if traffic else None,
        "traffic_over_algorithmic": round(traffic / cb, 3) if traffic else None,
        "timing": ("rocprofv3 kernel trace of a child bench's graph-replayed textureless steps "
                   "(last 16 dispatches of each region kernel); bytes: SURVEY 8(d) per group "
                   f"({per} B: position + 7 x {L} x {C} f16 gradients) at the child's groups "
                   "per step + the f32 table gradient")}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv=None):
    """`bench.py --gpus N` without a torch.distributed launcher: start N child
    processes (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their env,
    rendezvous on 127.0.0.1) and return the worst exit code.  Called before
    anything in this process touches the GPU, and it never exec()s: the
    children are fresh interpreters running this same file."""
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve()),
                                       *argv], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def launcher_selftest(args, rank, world):
    """CPU check of the N-rank launch (gloo): every rank joins, the all-reduced
    payload is the same everywhere and rank 0 prints the bench line's
    world-derived fields.  No GPU work."""
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(args.seed)               # identical replica init
    w = torch.randn(1024)
    g = torch.full((1024,), float(rank + 1))   # per-rank gradient
    dist.all_reduce(g)
    g /= world
    w -= 0.1 * g
    digest = torch.tensor([float(w.double().sum())], dtype=torch.float64)
    lo, hi = digest.clone(), digest.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "config": {"parallelism": f"dp{world}"},
                          "replicas_identical": bool(lo.item() == hi.item())}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launcher_selftest:
        return launcher_selftest(args, rank, world)
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)

    import _dfhip
    _dfhip.load()
    trainer, data = make_trainer(args.res, args.seed, rank, world, not args.two_pass_backward,
                                 graph=not args.eager, mock_sds=args.mock_sds)
    if args.module_path_child:
        trainer.native_step = False
        trainer.model.fused_field = False
    if args.shade != "albedo":
        trainer.pick_shading = (lambda k: (lambda: (k, 0.1)))(args.shade)

    def step():
        trainer.train_iteration(data.collate([0]))

    for _ in range(args.warmup):
        step()
    if args.module_path_child:
        # every sample-count bucket's graph captured now, none inside the
        # timed region (BucketedModuleStep)
        from nerf.graph import BucketedModuleStep
        seen = int(trainer.model.step_counter[:, 0].max().item())
        for g in trainer._graphs.values():
            if isinstance(g, BucketedModuleStep):
                g.precapture(2 * seen)
        torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # the timed region runs the product path: one graph replay per step (the
    # native step's graph holds the whole backward and, on one GPU, Adam)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    host_issue = time.perf_counter() - t0  # host done issuing (no sync inside the loop)
    barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    # samples per step: the renderer's per-step counts of the last min(16, K)
    # steps (read after the timed region; no copy inside the loop)
    last = min(16, args.steps)
    rows = [(trainer.model.local_step - 1 - i) % 16 for i in range(last)]
    samples = float(trainer.model.step_counter[rows, 0].float().mean().item())
    # the replicas after the timed region (every rank must hold the same
    # model: DDP's contract), and each rank's own samples per step
    identical, per_rank = replica_check(trainer, samples, world)
    kernels, timing = {}, None
    if not args.no_kernel_timing:
        kernels, timing = kernel_timing_pass(trainer, step, min(args.steps, 20))
    # host work per step with no queue back-pressure: one step issued on an
    # idle GPU (median of 16; the refresh step every 16 is the outlier)
    issue = []
    for _ in range(16):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        issue.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    host_cost = float(np.median(issue))

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
        "replicas_identical": identical,
        "samples_per_step_per_rank": per_rank,
        "host_issue_ms_per_step": round(host_issue / args.steps * 1e3, 3),
        "host_cost_ms_per_step": round(host_cost * 1e3, 3),
    }
    g0 = next(iter(trainer._graphs.values()), None)
    result["config"]["grad_exchange"] = "none (one rank)"
    if g0 is not None:
        result["config"]["optimizer_in_graph"] = bool(g0.optimizer_in_graph)
        nat0 = getattr(g0, "native", None)
        if world > 1:
            # one replay per step: RCCL all-reduce of the flat gradient bucket,
            # 1/world and GradScaler + Adam captured in the step graph
            result["config"]["grad_exchange"] = (
                "rccl all-reduce inside the replayed step graph"
                if nat0 is not None and nat0.dp_world is not None
                else "eager all-reduce after the replay")
    elif world > 1:
        result["config"]["grad_exchange"] = "eager flat all-reduce (rccl)"
    if "grad_allreduce" in kernels:
        # the exchange's time per step: HIP events around the same all-reduce +
        # 1/world launches in the eager twin of the replayed step (every rank
        # issues it; rank 0's events)
        result["grad_allreduce_us"] = kernels["grad_allreduce"]["avg_us"]
    if kernels:
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        kd = kernels[dom]
        traffic, note = (None, "skipped (--no-traffic or N > 1)")
        if world == 1 and not args.no_traffic:
            traffic, note = measure_traffic(dom, warmup=max(1, args.warmup + args.steps - 16))
        roof = {
            "kernel": dom, "bound": "hbm", "achieved": kd["achieved_GBs"], "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(kd["achieved_GBs"] / HBM_PEAK_GBS, 4),
            "traffic": traffic, "traffic_source": note,
            "traffic_by_kernel": MEASURE_TRAFFIC_DETAIL.get(dom),
            "avg_us": kd["avg_us"],
            "bytes_per_launch": kd["bytes_per_launch"],
            "timing": timing["note"] if timing else None}
        cm, tus = MEASURE_TRAFFIC_CHILD_M.get(dom), MEASURE_TRAFFIC_TRACE_US.get(dom)
        model = (timing or {}).get("models", {}).get(dom)
        if cm and tus and model:
            # ONE workload for bytes, time and traffic: the profiled child's
            # graph-replayed steps (its samples per step cm), its kernels'
            # rocprofv3 durations, its PMC bytes; the eager-twin event figures
            # of this process stay beside them
            base, per_row, live = model
            cb = base + (per_row * cm if live else 0)
            gbs = cb / (tus * 1e-6) / 1e9
            roof.update({
                "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                "avg_us": round(tus, 2), "bytes_per_launch": int(cb),
                "samples_per_step": round(cm, 1),
                "algorithmic_bytes_per_sample": round(cb / cm, 2),
                "traffic_per_sample": round(traffic / cm, 2) if traffic else None,
                "traffic_over_algorithmic": round(traffic / cb, 3) if traffic else None,
                "timing": ("rocprofv3 kernel trace of the child's graph-replayed steps "
                           "(last 16 dispatches of each region kernel), bytes from the "
                           "region's model at the child's samples per step"),
                "eager_twin": {"avg_us": kd["avg_us"], "bytes_per_launch": kd["bytes_per_launch"],
                               "achieved": kd["achieved_GBs"],
                               "frac": round(kd["achieved_GBs"] / HBM_PEAK_GBS, 4),
                               "samples_per_step": round(samples, 1),
                               "timing": timing["note"] if timing else None}})
        result["roofline"] = roof

        result["kernels"] = kernels
        result["step_roofline"] = step_roofline(kernels, timing["steps"], samples,
                                                rays_per_step, trainer)
        st_us = MEASURE_STEP_TRACE_US.get("step")
        if cm and st_us:
            # the same figure for the profiled child's replayed steps: every
            # region's byte model at the child's samples per step over the
            # rocprofv3 time of all kernels of a step
            models = timing.get("models", {})
            per_step = {k: v["launches"] / timing["steps"] for k, v in kernels.items()}
            sb = sum(per_step.get(k, 1.0) * (b + (pr * cm if lv else 0))
                     for k, (b, pr, lv) in models.items() if k in kernels)
            g = sb / (st_us * 1e-6) / 1e9
            result["step_roofline"]["replayed"] = {
                "samples_per_step": round(cm, 1), "bytes_per_step": int(sb),
                "kernel_us_per_step": round(st_us, 2), "achieved": round(g, 1),
                "frac": round(g / HBM_PEAK_GBS, 4),
                "note": "rocprofv3 kernel trace of the child's last 16 graph-replayed steps "
                        "(every kernel from a step prologue on: one density refresh, as in "
                        "every 16 steps of the timed region)"}
        result["kernel_timing"] = timing
    if world == 1 and not args.no_kernel_timing:
        result["field_mlp"] = field_mlp_report(trainer)
    if world == 1 and not args.no_alt_backward:
        # the other backward structure, same workload and launch mode: the
        # reference's two passes (sd.py:115 + utils.py:708) beside the fused
        # headline (or the fused one beside a --two-pass-backward headline)
        alt, alt_data = make_trainer(args.res, args.seed, rank, world, args.two_pass_backward,
                                     graph=not args.eager, mock_sds=args.mock_sds)
        for _ in range(args.warmup):
            alt.train_iteration(alt_data.collate([0]))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            alt.train_iteration(alt_data.collate([0]))
        torch.cuda.synchronize()
        key = "fused_ms_per_step" if args.two_pass_backward else "two_pass_ms_per_step"
        result[key] = round((time.perf_counter() - t0) / args.steps * 1e3, 3)
        del alt, alt_data
        torch.cuda.empty_cache()
    if world == 1 and not args.no_shading:
        # the steps after albedo_iters (utils.py:346-359): 20 % albedo, 40 %
        # textureless, 40 % lambertian (ambient 0.1), finite-difference normals
        shade = {}
        for kind in ("textureless", "lambertian"):
            tr, dat = make_trainer(args.res, args.seed, rank, world, True, graph=not args.eager,
                                   mock_sds=args.mock_sds)
            tr.pick_shading = (lambda k: (lambda: (k, 0.1)))(kind)
            for _ in range(args.warmup):
                tr.train_iteration(dat.collate([0]))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_iteration(dat.collate([0]))
            torch.cuda.synchronize()
            shade[f"{kind}_ms_per_step"] = round((time.perf_counter() - t0) / args.steps * 1e3, 3)
            del tr, dat
            torch.cuda.empty_cache()
        base = result["ms_per_step"] if not args.two_pass_backward else result.get(
            "fused_ms_per_step", result["ms_per_step"])
        shade["albedo_ms_per_step"] = base
        shade["schedule_ms_per_step"] = round(0.2 * base + 0.4 * shade["textureless_ms_per_step"]
                                              + 0.4 * shade["lambertian_ms_per_step"], 3)
        # main.py -O: albedo_iters 1000 of iters 10000, then the schedule
        shade["iters_weighted_ms_per_step"] = round(0.1 * base + 0.9 * shade["schedule_ms_per_step"],
                                                    3)
        shade["note"] = ("steps >= albedo_iters: 0.2 albedo + 0.4 textureless + 0.4 lambertian "
                         "(utils.py:346-359), native graph-replayed, fused backward; "
                         "iters_weighted: 0.1 albedo (albedo_iters 1000 of 10000) + 0.9 schedule")
        if not args.no_traffic:
            shade["roofline"] = shading_roofline(trainer, args)
        result["shading"] = shade
    if world == 1 and not args.no_module_path:
        result["module_path"] = module_path_leg(args)
    if world == 1 and not args.no_c5:
        result["c5"] = bench_c5(args, rank, world)
    if rank == 0 and world == 1 and not args.no_infer:
        result["inference"] = bench_inference(device, args.infer_res)
        result["inference_sphere"] = bench_inference(device, args.infer_res, occupancy="sphere")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.res, args.cpu_steps, args.c1_steps)
        result["gpu_vs_cpu"] = round(value / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
