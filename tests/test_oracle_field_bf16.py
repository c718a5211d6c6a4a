"""CPU checks of the bf16 restatement in oracle/field.py (the C5 option: the
field under bf16 autocast; no reference counterpart, the reference's kernels
dispatch f32 / f16 / f64 only).

* grid features: `encode_bf16` (bf16 table, f32 accumulation, one rounding)
  equals the f32 oracle encoding of the bf16-rounded table, rounded to bf16,
  and a lattice point reads exactly its corner's bf16 row;
* MLP: torch's own bf16 autocast (CPU: nn.Linear in bf16, f32 accumulation,
  ReLU on bf16 values) lands inside the oracle's bf16 windows everywhere and
  equals it bit for bit where the windows are closed; a wrong weight does not;
* backward: an independent autograd emulation of the bf16 graph stays inside
  the backward windows.
Reference semantics followed: nerf/network_grid.py:13-32,69-87 (the graph),
gridencoder.cu:75-178 (corner order and weights)."""
import numpy as np
import torch
import torch.nn as nn

import oracle
import oracle.field as of
from gridencoder.grid import level_offsets


def _table(seed, rows):
    return np.random.default_rng(seed).uniform(-0.5, 0.5, (rows, 2)).astype(np.float32)


def _levels():
    pls = np.exp2(np.log2(2048 / 16) / 15)
    return level_offsets(16, 2, 3, 16, pls, 16, False), float(np.log2(pls))


def test_encode_bf16_is_f32_encoding_rounded_once():
    offs, S = _levels()
    emb = _table(0, int(offs[-1]))
    xyz = np.random.default_rng(1).uniform(-1, 1, (4000, 3)).astype(np.float32)
    got = of.encode_bf16(xyz, 1.0, emb, offs, S, 16)
    x01 = ((xyz + np.float32(1)) / np.float32(2)).astype(np.float32)
    f32, _ = oracle.grid_encode_forward(x01, oracle.round_bf16(emb), offs, S, 16)
    assert np.array_equal(got, oracle.round_bf16(f32))
    # the f16 path (per-corner rounding) differs: the two modes are distinct
    assert not np.array_equal(got, of.encode(xyz, 1.0, emb, offs, S, 16).astype(np.float32))


def test_encode_bf16_lattice_point_reads_its_corner():
    offs, S = _levels()
    emb = _table(2, int(offs[-1]))
    # level 15 (scale 2047): x01 = 0.5 gives pos 0.5 * 2047 + 0.5 = 1024
    # exactly, so corner (1024, 1024, 1024) has weight 1 (z dropped, tiled)
    xyz = np.zeros((1, 3), np.float32)  # x01 = 0.5
    got = of.encode_bf16(xyz, 1.0, emb, offs, S, 16)
    scale = np.float32(np.float32(2.0 ** float(np.float32(15) * np.float32(S))) * np.float32(16)
                       - np.float32(1))
    assert float(scale) == 2047.0
    p = 1024
    smul = 2049  # res + 1
    row = int(offs[15]) + ((p + p * smul) & (int(offs[16] - offs[15]) - 1))  # z dropped
    want = oracle.round_bf16(emb[row])
    assert np.array_equal(got[0, 30:32], want)


def _case(seed, M=20000):
    r = np.random.default_rng(seed)
    x = oracle.round_bf16(r.uniform(-1, 1, (M, 32)).astype(np.float32))
    xyz = r.uniform(-1, 1, (M, 3)).astype(np.float32)
    lim = lambda k: 1 / np.sqrt(k)  # noqa: E731  (nn.Linear default init range)
    ws = [r.uniform(-lim(32), lim(32), (64, 32)), r.uniform(-lim(32), lim(32), 64),
          r.uniform(-lim(64), lim(64), (64, 64)), r.uniform(-lim(64), lim(64), 64),
          r.uniform(-lim(64), lim(64), (4, 64)), r.uniform(-lim(64), lim(64), 4)]
    return x, xyz, [w.astype(np.float32) for w in ws]


def _torch_bf16_mlp(x, ws):
    """The reference MLP (network_grid.py:13-32) under torch's bf16 autocast."""
    layers = nn.ModuleList([nn.Linear(32, 64), nn.Linear(64, 64), nn.Linear(64, 4)])
    with torch.no_grad():
        for i, lin in enumerate(layers):
            lin.weight.copy_(torch.from_numpy(ws[2 * i]))
            lin.bias.copy_(torch.from_numpy(ws[2 * i + 1]))
    h = torch.from_numpy(x).bfloat16()
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        for i, lin in enumerate(layers):
            h = lin(h)
            if i < 2:
                h = torch.relu(h)
    assert h.dtype == torch.bfloat16
    return h.float().numpy()


def test_forward_windows_hold_for_torch_bf16_autocast():
    x, xyz, ws = _case(3)
    with of.precision("bf16"):
        fo = of.field_forward(xyz, ws, x)
        fb = of.forward_bounds(fo, ws)
        tight = of.forward_bounds(fo, ws, acc_ulps=8)
    h = _torch_bf16_mlp(x, ws)
    dh = np.abs(h.astype(np.float64) - fo["h"].astype(np.float64))
    assert np.all(dh <= fb["dh"])
    closed = fb["dh"] == 0
    assert closed.mean() > 0.5
    assert np.array_equal(h[closed], fo["h"][closed])
    assert (tight["dh"] == 0).mean() > 0.5
    # bf16 windows are wider than f16's: the values are coarser
    assert np.all(np.abs(fo["h"]) < 64)


def test_forward_windows_catch_a_wrong_weight_bf16():
    x, xyz, ws = _case(4)
    with of.precision("bf16"):
        fo = of.field_forward(xyz, ws, x)
        fb = of.forward_bounds(fo, ws)
    bad = [w.copy() for w in ws]
    bad[2][5, 7] += 0.05  # one W2 entry off by ~5 % (bf16 keeps 8 bits)
    h = _torch_bf16_mlp(x, bad)
    dh = np.abs(h.astype(np.float64) - fo["h"].astype(np.float64))
    assert (dh > fb["dh"]).mean() > 0.02


def test_backward_windows_hold_bf16():
    x, xyz, ws = _case(5)
    r = np.random.default_rng(6)
    gs = r.normal(size=x.shape[0]).astype(np.float32) * 1e-2
    ga = oracle.round_bf16((r.normal(size=(x.shape[0], 3)) * 1e-2).astype(np.float32))
    with of.precision("bf16"):
        fo = of.field_forward(xyz, ws, x)
        fb = of.forward_bounds(fo, ws)
        bo = of.field_backward(fo, ws, gs, ga)
        bb = of.backward_bounds(fo, bo, ws, fb)
        ulp = of.ulp16(bo["d_enc"])
    w = [torch.from_numpy(oracle.round_bf16(v)).requires_grad_(True) for v in ws]
    xt = torch.from_numpy(x).requires_grad_(True)
    ste = lambda t: t + (t.bfloat16().float() - t).detach()  # noqa: E731  bf16 rounding
    a1 = torch.relu(ste(xt @ w[0].t() + w[1]))
    a2 = torch.relu(ste(a1 @ w[2].t() + w[3]))
    h = ste(a2 @ w[4].t() + w[5])
    sigma = torch.exp(h[:, 0] + torch.from_numpy(of.gaussian(xyz)))
    # sigmoid on the bf16 tensor, as under autocast: its backward uses the
    # saved bf16 output and rounds g (1 - y) y to bf16 (f32 opmath)
    alb = torch.sigmoid(h[:, 1:].bfloat16())
    for t in (h, a1, a2):
        t.register_hook(lambda g: g.bfloat16().float())
    loss = (sigma * torch.from_numpy(gs)).sum() + \
        (alb.float() * torch.from_numpy(ga)).sum()
    loss.backward()
    dx = xt.grad.bfloat16().float().numpy().astype(np.float64)
    dd = np.abs(dx - bo["d_enc"].astype(np.float64))
    rel = np.linalg.norm(dx - bo["d_enc"]) / np.linalg.norm(bo["d_enc"].astype(np.float64))
    assert rel < 2e-2
    assert (dd <= bb["d_enc"] + ulp).mean() > 0.99
