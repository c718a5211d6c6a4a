"""Run the sliced grid backward on one level range / parts setting (for PMC
passes): python tools/grid_bwd_case.py --first 0 --last 15 --parts 2 --reps 3"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests"), str(ROOT / "tools")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--last", type=int, default=15)
    ap.add_argument("--parts", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import _dfhip
    import _gridencoder
    import raymarching
    from scenes import march_inputs
    from gridencoder.grid import level_offsets
    from bench_kernels import timeit
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
    offs = offs_all[args.first:args.last + 2] - offs_all[args.first]
    H = int(round(16 * 2 ** (args.first * S))) if args.first else 16
    L = len(offs) - 1
    rows = int(offs[-1])
    g = (torch.randn(L, B, 2, device=dev) * 0.01).half()
    gemb = torch.empty(rows, 2, device=dev)
    parts = args.parts or _gridencoder.grid_backward_default_parts(rows, 2)
    partial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, 2, parts), device=dev)
    ot = T(offs.astype(np.int32))
    t = timeit(lambda: _gridencoder.grid_encode_backward_sliced(
        g, x01, ot, gemb, rows, B, 3, 2, L, S, H, 1, False, partial, parts), args.reps)
    print(f"B={B} levels={args.first}..{args.last} rows={rows} parts={parts} median_us={t:.1f}")


if __name__ == "__main__":
    main()
