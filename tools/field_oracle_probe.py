"""Probe: GPU fused field forward vs oracle/field.py in both accumulation
models (exact-rounded dot products / per-MFMA f32 rounding); prints the
fraction of samples whose outputs differ."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch
import _dfhip
import oracle.field as of
import test_gpu_field_oracle as t

_dfhip.load()
gpu = torch.device("cuda:0")
import _fieldmlp
for seed, sc in ((0, 0.5), (1, 1e-4), (2, 2.0)):
    enc_mod, layers = t._setup(gpu, seed, sc)
    xyzs, deltas, rays, M = t._march(gpu, 128, seed)
    S = float(np.log2(enc_mod.per_level_scale))
    ws = [p.detach().float().contiguous() for lin in layers for p in (lin.weight, lin.bias)]
    enc = torch.empty(M, 32, device=gpu, dtype=torch.half)
    sigma = torch.empty(M, device=gpu)
    albedo = torch.empty(M, 3, device=gpu, dtype=torch.half)
    _fieldmlp.grid_field_forward(xyzs, 1.0, enc_mod.embeddings.detach().half().contiguous(),
                                 enc_mod.offsets, S, 16, enc_mod.gridtype_id, False, ws, enc,
                                 sigma, albedo, None)
    x = t._unperm(enc.cpu().numpy())
    s_g, a_g = sigma.cpu().numpy(), albedo.cpu().numpy()
    for chunk in (None, 32, 16, 8):
        fo = of.field_forward(xyzs.cpu().numpy(), [w.cpu().numpy() for w in ws], x, chunk)
        ds = np.abs(s_g.astype(np.float64) / fo["sigma"] - 1)
        da = (a_g != fo["albedo"]).any(1)
        print(f"seed {seed} scale {sc} chunk {chunk}: M={M} sigma rel>2e-7 {np.mean(ds > 2e-7):.3e} "
              f"max {ds.max():.2e}; albedo differ {da.mean():.3e}", flush=True)
