"""Probe: where the GPU feature gradients leave the oracle's windows, print
the exact sum, its distance to the nearest f16 rounding boundary in units of
sum|terms| * 2^-24, and whether the row's dz1 operands hold f16 subnormals."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch
import _dfhip
import oracle
import oracle.field as of
import test_gpu_field_oracle as t
import _fieldmlp
import _raymarching

_dfhip.load()
gpu = torch.device("cuda:0")
enc_mod, layers = t._setup(gpu, 0, 0.5)
xyzs, deltas, rays, M = t._march(gpu, 128, 0)
N = rays.shape[0]
S = float(np.log2(enc_mod.per_level_scale))
ws = [p.detach().float().contiguous() for lin in layers for p in (lin.weight, lin.bias)]
ws_np = [w.cpu().numpy() for w in ws]
enc = torch.empty(M, 32, device=gpu, dtype=torch.half)
sigma = torch.empty(M, device=gpu)
albedo = torch.empty(M, 3, device=gpu, dtype=torch.half)
_fieldmlp.grid_field_forward(xyzs, 1.0, enc_mod.embeddings.detach().half().contiguous(),
                             enc_mod.offsets, S, 16, enc_mod.gridtype_id, False, ws, enc, sigma,
                             albedo, None)
x16 = t._unperm(enc.cpu().numpy())
for scale in (1e-5, 1e-6):
    g = torch.Generator(device="cpu").manual_seed(10)
    gs = (torch.randn(M, generator=g) * scale).to(gpu)
    grgb = (torch.randn(M, 3, generator=g) * scale).to(gpu)
    d_enc = torch.empty(16, M, 2, device=gpu, dtype=torch.half)
    partial = torch.empty(_fieldmlp.backward_parts(M) * _fieldmlp.params_count(), device=gpu)
    grads = [torch.empty_like(w) for w in ws]
    _fieldmlp.grid_field_backward(enc, xyzs, 1.0, ws, gs, grgb, d_enc, partial, grads,
                                  enc_mod.offsets, 0, S, 16, enc_mod.gridtype_id, False, None,
                                  None, 1, None)
    fo = of.field_forward(xyzs.cpu().numpy(), ws_np, x16)
    fb = of.forward_bounds(fo, ws_np, acc_ulps=8)
    bo = of.field_backward(fo, ws_np, gs.cpu().numpy(), grgb.cpu().numpy().astype(np.float16))
    bb = of.backward_bounds(fo, bo, ws_np, fb, acc_ulps=None)
    fbr = of.forward_bounds(fo, ws_np, acc_ulps=None)
    bbr = of.backward_bounds(fo, bo, ws_np, fbr, acc_ulps=None)
    got = d_enc.cpu().numpy().transpose(1, 0, 2).reshape(M, 32).astype(np.float64)
    want = bo["d_enc"].astype(np.float64)
    dd = np.abs(got - want)
    bad = dd > bb["d_enc"]
    print(f"scale {scale}: violations {bad.sum()} of {bad.size}; differing {(dd > 0).mean():.3e}; "
          f"with order-free forward windows: {(dd > bbr['d_enc']).sum()}")
    if bad.any():
        r, c = np.nonzero(bad)
        dz1 = bo["dz1"].astype(np.float64)
        w1 = of.r16(ws_np[0]).astype(np.float64)
        for i in range(min(12, len(r))):
            m, k = r[i], c[i]
            terms = dz1[m] * w1[:, k]
            ex = bo["dX"][m, k]
            sub = np.sum((np.abs(bo["dz1"][m]) < 6.1e-5) & (bo["dz1"][m] != 0))
            print(f"  m {m} k {k}: exact {ex:.6e} got {got[m, k]:.6e} want {want[m, k]:.6e} "
                  f"sum|t| {np.abs(terms).sum():.3e} subnormal dz1 operands {sub}, "
                  f"window {bb['d_enc'][m, k]:.2e}")
        # flush-to-zero model of subnormal f16 MFMA operands
        def ftz(a):
            a = a.astype(np.float64)
            return np.where(np.abs(a) < 2.0 ** -14, 0.0, a)
        w = [of.r16(v).astype(np.float64) for v in ws_np]
        dO = ftz(bo["dO"])
        dz2 = np.where(fo["a2"] > 0, of.r16(dO @ w[4]), 0)
        dz1 = np.where(fo["a1"] > 0, of.r16(ftz(dz2) @ w[2]), 0)
        dx = of.r16(ftz(dz1) @ w[0]).astype(np.float64)
        print(f"  FTZ model: equal to GPU {(dx == got).mean():.6f}; exact model "
              f"{(want == got).mean():.6f}")
        vals = np.abs(want[bad])
        print(f"  |want| of violations: min {vals.min():.3e} max {vals.max():.3e}; "
              f"subnormal-range fraction {(vals < 6.1e-5).mean():.3f}")
