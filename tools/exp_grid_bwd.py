"""Experiment: where does the sliced grid backward spend its time?
Times the kernel on (a) coarse levels only, (b) fine levels only, (c) all."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests"), str(ROOT / "tools")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_kernels import timeit  # noqa: E402


def main():
    import _dfhip
    import _gridencoder
    import raymarching
    from scenes import march_inputs
    from gridencoder.grid import level_offsets
    _dfhip.load()
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    rays_o, rays_d, nears, fars, noises, bf = march_inputs(128, 128, seed=0, radius=0.56, noise=0.0)
    o, d, ne, fa, b = map(T, (rays_o, rays_d, nears, fars, bf))
    counter = torch.zeros(2, dtype=torch.int32, device=dev)
    xyzs, _, _, _ = raymarching.march_rays_train(o, d, 1.0, b, 1, 128, ne, fa, counter, -1, True,
                                                 128, True, 0.0, 512)
    B = xyzs.shape[0]
    x01 = ((xyzs + 1) / 2).contiguous()
    pls = np.exp2(np.log2(2048 / 16) / 15)
    S = float(np.log2(pls))
    offs_all = level_offsets(16, 2, 3, 16, pls, 16, False)
    out = {"B": B}
    cases = {
        "coarse_0_2": (offs_all[:4], 16),
        "mid_3_8": (offs_all[3:10] - offs_all[3], None),
        "fine_9_15": (offs_all[9:] - offs_all[9], None),
        "all": (offs_all, 16),
    }
    for name, (offs, H) in cases.items():
        L = len(offs) - 1
        first = {"coarse_0_2": 0, "mid_3_8": 3, "fine_9_15": 9, "all": 0}[name]
        # levels first..first+L-1 re-based to 0: same scales via a shifted base resolution
        Sx = S
        Hx = H if H is not None else int(round(16 * 2 ** (first * S)))
        rows = int(offs[-1])
        g = (torch.randn(L, B, 2, device=dev) * 0.01).half()
        gemb = torch.empty(rows, 2, device=dev)
        for parts in (1, 2, 8):
            partial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, 2, parts), device=dev)
            t = timeit(lambda: _gridencoder.grid_encode_backward_sliced(
                g, x01, T(offs.astype(np.int32)), gemb, rows, B, 3, 2, L, Sx, Hx, 1, False, partial,
                parts), 10)
            out[f"{name}_p{parts}_us"] = round(t, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
