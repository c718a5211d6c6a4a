"""Debug: the binned stencil backward, walk mode 0, alone in a fresh process,
against the f64 oracle; per-level error report and the plan's image slots."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch
import _dfhip
import _gridencoder
import oracle
from test_gpu_encoders import _grid_consts, _samples, T

gpu = torch.device("cuda")
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
opts = _gridencoder.BinnedOpts(walk_mode=mode)
offs, S, _ = _grid_consts()
rows = int(offs[-1])
cap, m, eps = 5000, 4321, 1e-2
x = (_samples(cap, 63, edge=False) * 2 - 1).astype(np.float32)
x[:40, 1] = np.float32(1.0)
xt = T(x, gpu)
m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
x7 = torch.empty(7 * cap, 3, device=gpu)
m7 = torch.zeros(1, dtype=torch.int32, device=gpu)
_dfhip.call("dfhip_shading_stencil", xt.data_ptr(), m_dev.data_ptr(), cap, eps, 1.0,
            x7.data_ptr(), m7.data_ptr(), _dfhip.stream())
g7 = (torch.randn(16, 7 * cap, 2, generator=torch.Generator().manual_seed(64)) * 0.1)
g7 = g7.half().to(gpu)
ne, nc, npf = _gridencoder.grid_backward_binned_scratch(cap, offs, 16, 2, opts, group=7)
ent = torch.zeros(ne, dtype=torch.int32, device=gpu)
cnt = torch.zeros(nc, dtype=torch.int32, device=gpu)
part = torch.full((npf,), 777.0, device=gpu)
gemb = torch.full((rows, 2), float("nan"), device=gpu)
_gridencoder.binned_launcher(g7, xt, 1.0, T(offs, gpu), offs, gemb, cap, m_dev, 3, 2, 16,
                             S, 16, 1, False, ent, cnt, part, stencil_eps=eps, opts=opts)()
torch.cuda.synchronize()
x01 = ((x7[:7 * m].cpu().numpy() + np.float32(1)) / np.float32(2)).astype(np.float32)
gl = g7[:, :7 * m].float().cpu().numpy()
want = oracle.grid_encode_backward(gl, x01, offs, 2, S, 16, gridtype=1, blc=False)
got = gemb.double().cpu().numpy()
bad = ~np.isclose(got, want, rtol=1e-5, atol=1e-7 * np.abs(want).max())
print("scratch", ne, nc, npf, "tile", _gridencoder.grid_backward_binned_tile(opts, 7))
print("bad rows", int(bad.any(1).sum()), "of", rows, "nan", int(np.isnan(got).sum()),
      "777-ish", int((np.abs(got - 777) < 1e-3).sum()))
for l in range(16):
    sl = slice(offs[l], offs[l + 1])
    print(f"level {l}: bad {int(bad[sl].any(1).sum())} / {offs[l + 1] - offs[l]}")
