"""Per-kernel microbenchmark on a realistic C2 workload (one 128x128 view of a
radius-0.56 occupied sphere, ~0.7 M samples): HIP-event median times of the
hot-path kernels and their algorithmic GB/s.  Prints one JSON object.

    python tools/bench_kernels.py [--reps 20] [--only grid_bwd]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timeit(fn, reps):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import _dfhip
    import _gridencoder
    import _raymarching
    import raymarching
    from scenes import march_inputs
    from gridencoder.grid import level_offsets
    _dfhip.load()
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731

    rays_o, rays_d, nears, fars, noises, bf = march_inputs(128, 128, seed=0, radius=0.56,
                                                           noise=0.0)
    o, d, ne, fa, no, b = map(T, (rays_o, rays_d, nears, fars, noises, bf))
    n = o.shape[0]
    counter = torch.zeros(2, dtype=torch.int32, device=dev)
    xyzs, dirs, deltas, rays = raymarching.march_rays_train(o, d, 1.0, b, 1, 128, ne, fa, counter,
                                                            -1, True, 128, True, 0.0, 512)
    B = xyzs.shape[0]
    out = {"samples": B, "rays": n}

    def want(name):
        return not args.only or args.only in name

    # -------------------------------------------------------------- march
    if want("march"):
        rays2 = torch.empty(n, 3, dtype=torch.int32, device=dev)
        bs = torch.empty(_raymarching.march_rays_train_scratch_ints(n), dtype=torch.int32, device=dev)
        cap = n * 512
        bx = torch.empty(cap, 3, device=dev)
        bd = torch.empty(cap, 3, device=dev)
        bl = torch.empty(cap, 2, device=dev)

        def count():
            counter.zero_()
            _raymarching.march_rays_train_count(o, d, b, 1.0, 0.0, 512, n, 1, 128, ne, fa, rays2,
                                                counter, no, bs)

        def emit():
            _raymarching.march_rays_train_emit(o, d, b, 1.0, 0.0, 512, n, 1, 128, cap, ne, fa, bx,
                                               bd, bl, rays2, no, bs, 128)
        count()
        out["march_count_us"] = timeit(count, args.reps)
        out["march_emit_us"] = timeit(emit, args.reps)

    # -------------------------------------------------------------- grid
    pls = np.exp2(np.log2(2048 / 16) / 15)
    offs = T(level_offsets(16, 2, 3, 16, pls, 16, False))
    rows = int(offs[-1])
    S = float(np.log2(pls))
    emb = (torch.rand(rows, 2, device=dev) - 0.5).half()
    x01 = ((xyzs + 1) / 2).contiguous()
    feats = torch.empty(B, 32, dtype=torch.float16, device=dev)
    if want("grid_fwd"):
        t = timeit(lambda: _gridencoder.grid_encode_forward_blc(x01, emb, offs, feats, B, 3, 2, 16,
                                                                S, 16, None, 1, False), args.reps)
        out["grid_fwd_us"] = t
        out["grid_fwd_GBs"] = B * (12 + 64) / t / 1e3
    g = (torch.randn(B, 32, device=dev) * 0.01).half()
    if want("grid_bwd"):
        glbc = torch.empty(16, B, 2, dtype=g.dtype, device=dev)
        out["grid_bwd_transpose_torch_us"] = timeit(
            lambda: g.view(B, 16, 2).transpose(0, 1).contiguous(), args.reps)
        out["grid_bwd_transpose_us"] = timeit(
            lambda: _gridencoder.grid_grad_blc_to_lbc(g, glbc, B, 16, 2), args.reps)
        gemb = torch.empty(rows, 2, device=dev)
        dflt = _gridencoder.grid_backward_default_parts(rows, 2)
        out["grid_bwd_default_parts"] = dflt
        for parts in sorted({2, 4, dflt, 6, 8, 12, 16, 24}):
            partial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, 2, parts),
                                  device=dev)
            t = timeit(lambda: _gridencoder.grid_encode_backward_sliced(
                glbc, x01, offs, gemb, rows, B, 3, 2, 16, S, 16, 1, False, partial, parts),
                args.reps)
            out[f"grid_bwd_sliced_p{parts}_us"] = t
        gatom = torch.zeros(rows, 2, dtype=torch.float16, device=dev)
        out["grid_bwd_atomic_f16_us"] = timeit(lambda: _gridencoder.grid_encode_backward_blc(
            g, x01, offs, gatom, B, 3, 2, 16, S, 16, None, None, 1, False), max(3, args.reps // 4))

    # -------------------------------------------------------------- field MLP
    if want("field"):
        import _fieldmlp
        enc16 = (torch.randn(B, 32, device=dev) * 0.5).half()
        xw = (torch.rand(B, 3, device=dev) * 2 - 1)
        torch.manual_seed(0)
        ws = [torch.randn(64, 32, device=dev) * 0.2, torch.randn(64, device=dev) * 0.1,
              torch.randn(64, 64, device=dev) * 0.15, torch.randn(64, device=dev) * 0.1,
              torch.randn(4, 64, device=dev) * 0.15, torch.randn(4, device=dev) * 0.1]
        sig = torch.empty(B, device=dev)
        alb = torch.empty(B, 3, device=dev, dtype=torch.half)
        out["field_fwd_us"] = timeit(lambda: _fieldmlp.field_mlp_forward(enc16, xw, ws, sig, alb),
                                     args.reps)
        gsig = torch.randn(B, device=dev)
        galb = torch.randn(B, 3, device=dev).half()
        denc = torch.empty(16, B, 2, device=dev, dtype=torch.half)
        part = torch.empty(_fieldmlp.backward_parts(B) * _fieldmlp.params_count(), device=dev)
        grads = [torch.empty_like(w) for w in ws]
        out["field_bwd_us"] = timeit(lambda: _fieldmlp.field_mlp_backward(
            enc16, xw, ws, gsig, galb, denc, part, grads), args.reps)

    # -------------------------------------------------------------- fused grid field
    if want("fused"):
        import _fieldmlp
        torch.manual_seed(0)
        mlp = [torch.randn(64, 32, device=dev) * 0.2, torch.randn(64, device=dev) * 0.1,
               torch.randn(64, 64, device=dev) * 0.15, torch.randn(64, device=dev) * 0.1,
               torch.randn(4, 64, device=dev) * 0.15, torch.randn(4, device=dev) * 0.1]
        encf = torch.empty(B, 32, dtype=torch.float16, device=dev)
        sigf = torch.empty(B, device=dev)
        albf = torch.empty(B, 3, dtype=torch.float16, device=dev)
        out["fused_field_fwd_us"] = timeit(lambda: _fieldmlp.grid_field_forward(
            xyzs, 1.0, emb, offs, S, 16, 1, False, mlp, encf, sigf, albf, None), args.reps)

    # -------------------------------------------------------------- composite
    if want("composite"):
        sig = torch.rand(B, device=dev) * 30
        rgb = torch.rand(B, 3, device=dev)
        ws = torch.empty(n, device=dev)
        dep = torch.empty(n, device=dev)
        img = torch.empty(n, 3, device=dev)
        out["composite_fwd_us"] = timeit(lambda: _raymarching.composite_rays_train_forward(
            sig, rgb, deltas, rays, B, n, 1e-4, ws, dep, img), args.reps)
        gs = torch.empty(B, device=dev)
        gc = torch.empty(B, 3, device=dev)
        gws = torch.randn(n, device=dev)
        gim = torch.randn(n, 3, device=dev)
        out["composite_bwd_us"] = timeit(lambda: _raymarching.composite_rays_train_backward_dense(
            gws, gim, sig, rgb, deltas, rays, ws, img, B, n, 1e-4, gs, gc), args.reps)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}))


if __name__ == "__main__":
    main()
