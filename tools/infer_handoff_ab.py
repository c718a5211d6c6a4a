"""A/B of the C4 renderer's straggler hand-off (csrc/render.hip): the bench's
800 x 800 frame (R0 grid occupancy and R1 sphere), frames timed with events for
each handoff_lanes value, the variants interleaved `--rounds` times on one box;
outputs checked bit-identical across variants.
    python tools/infer_handoff_ab.py [--values 0,8,16,24,32] [--reps 10]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def scene(occupancy, res, dev):
    import bench
    import main as m
    from nerf.network_grid import NeRFNetwork
    from nerf.provider import NeRFDataset
    opt = m.parse_opt(["--text", "a hamburger", "-O", "--h", str(res), "--w", str(res)])
    torch.manual_seed(1)
    model = NeRFNetwork(opt).to(dev)
    with torch.no_grad():
        model.encoder.embeddings.uniform_(-0.5, 0.5)
    with torch.autocast("cuda", dtype=torch.float16):
        for _ in range(3):
            model.update_extra_state()
    if occupancy == "sphere":
        bench.sphere_occupancy_(model)
    model.eval()
    data = NeRFDataset(opt, device=dev, type="test", H=res, W=res, size=8).collate([1])
    return model, opt, data


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--values", default="0,8,16,24,32")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--res", type=int, default=800)
    args = ap.parse_args()
    dev = torch.device("cuda")
    vals = [int(v) for v in args.values.split(",")]
    for occ in ("grid", "sphere"):
        model, opt, data = scene(occ, args.res, dev)

        def frame():
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
                return model.render(data["rays_o"], data["rays_d"], staged=True, perturb=False,
                                    light_d=None, ambient_ratio=1.0, shading="albedo",
                                    force_all_rays=True, bg_color=None, **vars(opt))
        ref, times = None, {v: [] for v in vals}
        for _ in range(args.rounds):
            for v in vals:
                model.infer_handoff = v
                for _ in range(2):
                    out = frame()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    frame()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.reps)
                got = [out[k].float().cpu().numpy() for k in ("image", "depth", "weights_sum")]
                if ref is None:
                    ref = got
                else:
                    for a, b in zip(ref, got):
                        assert np.array_equal(a, b), f"handoff {v}: outputs differ"
                work = model.last_infer_work.cpu().numpy().view(np.uint32)
                samples = int(work[1]) + (int(work[2]) << 32)
                print(f"{occ} handoff={v:3d} ms_per_frame={times[v][-1]:.3f} "
                      f"handed_off={int(work[3])} samples={samples}", flush=True)
        for v in vals:
            print(f"SUMMARY {occ} handoff={v:3d} ms_per_frame min {min(times[v]):.3f} "
                  f"mean {sum(times[v]) / len(times[v]):.3f}", flush=True)


if __name__ == "__main__":
    main()
