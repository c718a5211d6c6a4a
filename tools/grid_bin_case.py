"""Binned grid backward (csrc/gridbin.hip) on the samples of a real 128x128
march, per level range (timing study / PMC passes):
    python tools/grid_bin_case.py [--reps 5] [--ranges 0-15,0-2,3-8,9-15]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests"),
          str(ROOT / "tools")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ranges", default="0-15,0-2,3-8,9-15")
    ap.add_argument("--modes", default="-1", help="walk modes (dfhip_binned_opts.walk_mode)")
    args = ap.parse_args()
    import _dfhip
    import _gridencoder
    import raymarching
    from bench_kernels import timeit
    from gridencoder.grid import level_offsets
    from scenes import march_inputs
    _dfhip.load()
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    rays_o, rays_d, nears, fars, _, bf = march_inputs(128, 128, seed=0, radius=0.56, noise=0.0)
    o, d, ne, fa, b = map(T, (rays_o, rays_d, nears, fars, bf))
    counter = torch.zeros(2, dtype=torch.int32, device=dev)
    xyzs, _, _, _ = raymarching.march_rays_train(o, d, 1.0, b, 1, 128, ne, fa, counter, -1, True,
                                                 128, True, 0.0, 512)
    B = xyzs.shape[0]
    x01 = ((xyzs + 1) / 2).contiguous()
    pls = np.exp2(np.log2(2048 / 16) / 15)
    S = float(np.log2(pls))
    offs_all = level_offsets(16, 2, 3, 16, pls, 16, False)
    for rng in args.ranges.split(","):
        first, last = (int(v) for v in rng.split("-"))
        offs = (offs_all[first:last + 2] - offs_all[first]).astype(np.int32)
        H = 16 * 2 ** (first * S)
        L = len(offs) - 1
        rows = int(offs[-1])
        g = (torch.randn(L, B, 2, device=dev) * 0.01).half()
        ot = T(offs)
        ref = None
        for mode in (int(v) for v in args.modes.split(",")):
            opts = _gridencoder.BinnedOpts(walk_mode=mode)
            gemb = torch.empty(rows, 2, device=dev)
            Hr = int(round(H))  # H rounded: representative cell sizes
            ne_, nc, npf = _gridencoder.grid_backward_binned_scratch(B, offs, L, 2, opts)
            ent = torch.empty(ne_, dtype=torch.int32, device=dev)
            cnt = torch.empty(nc, dtype=torch.int32, device=dev)
            part = torch.empty(npf, device=dev)
            # S and H of the sub-range: level l' = l - first has scale 2^(l*S)*16 - 1
            t = timeit(lambda: _gridencoder.grid_encode_backward_binned(
                g, x01, 0.0, ot, offs, gemb, B, None, 3, 2, L, S, Hr, 1, False, ent, cnt,
                part, opts=opts), args.reps)
            torch.cuda.synchronize()
            if ref is None:
                ref = gemb.clone()
            err = float(((gemb - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item())
            print(f"B={B} levels={first}..{last} rows={rows} mode={mode} median_us={t:.1f} "
                  f"max_rel_diff_vs_first={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
