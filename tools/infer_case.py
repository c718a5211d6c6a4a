"""C4 fused inference renderer (csrc/render.hip k_render_infer) on the bench's
800x800 scene (tools for timing studies / PMC passes):
    python tools/infer_case.py [--reps 10] [--res 800]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--profile", action="store_true",
                    help="per-wave phase cycles of k_render_infer (dfhip_render_rays_infer_prof)")
    ap.add_argument("--strips", action="store_true",
                    help="64-ray row strips as queue chunks (default: 8 x 8 tiles, renderer.infer_tile_w)")
    ap.add_argument("--serial-bg", action="store_true",
                    help="background net after the render (renderer.infer_overlap_bg = False)")
    ap.add_argument("--order", type=int, default=1,
                    help="queue order: 0 pixel, 1 line distance, 2 occupied cells (renderer.infer_order)")
    ap.add_argument("--dump", default="", help="save the per-wave records (.npy; last row: prof[:16])")
    ap.add_argument("--sphere", action="store_true", help="analytic sphere occupancy (R1)")
    args = ap.parse_args()
    import main as m
    from nerf.network_grid import NeRFNetwork
    from nerf.provider import NeRFDataset
    dev = torch.device("cuda")
    opt = m.parse_opt(["--text", "a hamburger", "-O", "--h", str(args.res), "--w", str(args.res)])
    torch.manual_seed(1)
    model = NeRFNetwork(opt).to(dev)
    with torch.no_grad():
        model.encoder.embeddings.uniform_(-0.5, 0.5)
    with torch.autocast("cuda", dtype=torch.float16):
        for _ in range(3):
            model.update_extra_state()
    if args.sphere:
        import bench
        bench.sphere_occupancy_(model)
    model.eval()
    model.native_infer = True
    model.infer_tile_w = 0 if args.strips else args.res
    model.infer_overlap_bg = not args.serial_bg
    model.infer_order = args.order
    data = NeRFDataset(opt, device=dev, type="test", H=args.res, W=args.res, size=8).collate([1])

    def frame():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            return model.render(data["rays_o"], data["rays_d"], staged=True, perturb=False,
                                light_d=None, ambient_ratio=1.0, shading="albedo",
                                force_all_rays=True, bg_color=None, **vars(opt))
    for _ in range(3):
        out = frame()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        frame()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    img = out["image"].float()
    print(f"res={args.res} ms_per_frame={ms:.3f} image_mean={float(img.mean()):.6f} "
          f"ws_mean={float(out['weights_sum'].float().mean()):.6f}", flush=True)
    if args.profile:
        import functools
        import _fieldmlp
        W = 8192  # per-wave records
        prof = torch.zeros(16 + 16 * W, dtype=torch.int64, device=dev)
        prof[6] = prof[7] = -1  # UINT64_MAX (atomicMin slots)
        prof[10] = W
        plain = _fieldmlp.render_rays_infer
        _fieldmlp.render_rays_infer = functools.partial(plain, prof=prof)
        try:
            frame()
        finally:
            _fieldmlp.render_rays_infer = plain
        torch.cuda.synchronize()
        p = prof.cpu().tolist()
        tot = sum(p[:4])
        print("phase cycles (summed over waves): " + ", ".join(
            f"{n} {v / tot:.3f}" for n, v in zip(("refill", "march", "field", "composite"), p[:4]))
            + f"; rounds {p[4]}, tiles {p[5]}, cycles/round {tot / max(1, p[4]):.0f}, "
            f"field cycles/tile {p[2] / max(1, p[5]):.0f}", flush=True)
        span = max(1, p[8] - p[6])
        waves = p[9] / span  # mean resident waves over the kernel's span
        print(f"wall span {span / 100:.1f} us (100 MHz ticks); queue dry after "
              f"{(p[7] - p[6]) / 100:.1f} us ({(p[7] - p[6]) / span:.3f} of the span); "
              f"mean resident waves {waves:.0f}", flush=True)
        import numpy as np
        rec = prof[16:].view(W, 16).cpu().numpy().astype(np.int64)
        rec = rec[rec[:, 0] != 0]
        if args.dump:
            np.save(args.dump, np.concatenate([rec, np.array([p[:16]], dtype=np.int64)]))
        t0, dry0 = p[6], p[7]
        start = (rec[:, 0] - t0) / 100.0
        end = (rec[:, 2] - t0) / 100.0
        sawdry = rec[:, 1] != 0
        dry = np.where(sawdry, (rec[:, 1] - t0) / 100.0, np.nan)
        held = rec[:, 3] & 0xFF
        rdry = (rec[:, 3] & 0xFFFFFFFF) >> 8
        rounds = rec[:, 3] >> 32
        q = [0, 10, 25, 50, 75, 90, 99, 100]
        def pct(a):
            a = a[~np.isnan(a)]
            return " ".join(f"{v:.0f}" for v in np.percentile(a, q)) if a.size else "-"
        print(f"waves {len(rec)} (percentiles {q}, us from the first start)", flush=True)
        print(f"  start       {pct(start)}", flush=True)
        print(f"  first dry   {pct(dry)}  (waves never seeing it: {int((~sawdry).sum())})", flush=True)
        print(f"  end         {pct(end)}", flush=True)
        print(f"  end - dry   {pct(end - dry)}", flush=True)
        print(f"  held at dry {pct(held[sawdry].astype(float))}", flush=True)
        print(f"  rounds      {pct(rounds.astype(float))}", flush=True)
        print(f"  rounds after dry {pct(np.where(sawdry, rounds - rdry, np.nan).astype(float))}", flush=True)
        print(f"  max marched {pct(rec[:, 4].astype(float))}", flush=True)
        print(f"  max taken   {pct(rec[:, 6].astype(float))}", flush=True)
        print(f"  samples     {pct(rec[:, 5].astype(float))}", flush=True)
        print(f"  rays        {pct(rec[:, 7].astype(float))}", flush=True)
        slow = end >= np.percentile(end, 99)
        print(f"  slowest 1%: samples {pct(rec[slow, 5].astype(float))} max marched "
              f"{pct(rec[slow, 4].astype(float))} rays {pct(rec[slow, 7].astype(float))} "
              f"rounds {pct(rounds[slow].astype(float))}", flush=True)
        late = end > (dry0 - t0) / 100.0 + 0.5 * ((p[8] - dry0) / 100.0)
        print(f"  waves ending in the last half of the drain: {int(late.sum())}; their held "
              f"at dry {pct(held[late & sawdry].astype(float))}, rounds after dry "
              f"{pct((rounds - rdry)[late & sawdry].astype(float))}", flush=True)


if __name__ == "__main__":
    main()
