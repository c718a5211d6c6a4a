"""CPU checks of oracle/field.py (the f16-autocast field restatement and its
error windows): an independent f32-accumulating emulation of the same graph
(torch float32 GEMMs on the f16 values, rounded to f16 per layer, as autocast
does — network_grid.py:13-32,76-87) must land inside the oracle's windows
everywhere, equal the oracle bit for bit where the windows are closed, and the
backward must do the same.  A perturbed result (one wrong weight) must not."""
import numpy as np
import torch

import oracle.field as of


def _f32_field(x16, xyz, ws, order=1):
    """Forward + backward with f32 accumulation in torch (CPU), a different
    summation order than the oracle's exact sums (order=-1 reverses k)."""
    w1, b1, w2, b2, w3, b3 = (torch.from_numpy(of.r16(w).astype(np.float32)) for w in ws)

    def lin(a, w, b):
        if order < 0:
            a, w = a.flip(1), w.flip(1)
        return (a @ w.t() + b).half().float()

    x = torch.from_numpy(x16.astype(np.float32))
    a1 = torch.relu(lin(x, w1, b1))
    a2 = torch.relu(lin(a1, w2, b2))
    h = lin(a2, w3, b3)
    y = h[:, 0] + torch.from_numpy(of.gaussian(xyz))
    return x, a1, a2, h, torch.exp(y), torch.sigmoid(h[:, 1:]).half().float(), y


def _case(seed, M=20000):
    r = np.random.default_rng(seed)
    x16 = (r.uniform(-1, 1, (M, 32))).astype(np.float16)
    xyz = r.uniform(-1, 1, (M, 3)).astype(np.float32)
    lim = lambda k: 1 / np.sqrt(k)  # noqa: E731  (nn.Linear default init range)
    ws = [r.uniform(-lim(32), lim(32), (64, 32)), r.uniform(-lim(32), lim(32), 64),
          r.uniform(-lim(64), lim(64), (64, 64)), r.uniform(-lim(64), lim(64), 64),
          r.uniform(-lim(64), lim(64), (4, 64)), r.uniform(-lim(64), lim(64), 4)]
    return x16, xyz, [w.astype(np.float32) for w in ws]


def test_forward_windows_hold_for_f32_accumulation():
    for seed, order in ((0, 1), (1, -1)):
        x16, xyz, ws = _case(seed)
        fo = of.field_forward(xyz, ws, x16)
        fb = of.forward_bounds(fo, ws)
        _, _, _, h, sigma, alb, _ = _f32_field(x16, xyz, ws, order)
        dh = np.abs(h.numpy().astype(np.float64) - fo["h"].astype(np.float64))
        assert np.all(dh <= fb["dh"])
        dlog = np.abs(np.log(sigma.double().numpy()) - np.log(fo["sigma"].astype(np.float64)))
        assert np.all(dlog <= fb["dlog_sigma"])
        da = np.abs(alb.numpy().astype(np.float64) - fo["albedo"].astype(np.float64))
        assert np.all(da <= fb["dalbedo"])
        # closed windows -> bit-exact
        closed = fb["dh"] == 0
        assert np.array_equal(h.numpy()[closed], fo["h"].astype(np.float32)[closed])
        # the rigorous any-order windows are wide (64-term sums); the MFMA
        # model's few-rounding windows are tight and still hold for a
        # blocked f32 GEMM
        tight = of.forward_bounds(fo, ws, acc_ulps=8)
        assert np.all(dh <= tight["dh"])
        assert (tight["dh"] == 0).all(1).mean() > 0.3


def test_forward_windows_catch_a_wrong_weight():
    x16, xyz, ws = _case(2)
    fo = of.field_forward(xyz, ws, x16)
    fb = of.forward_bounds(fo, ws)
    bad = [w.copy() for w in ws]
    bad[2][5, 7] += 0.01  # one W2 entry off by ~1 %
    _, _, _, h, _, _, _ = _f32_field(x16, xyz, bad)
    dh = np.abs(h.numpy().astype(np.float64) - fo["h"].astype(np.float64))
    assert (dh > fb["dh"]).mean() > 0.05


def test_backward_windows_hold_for_f32_accumulation():
    x16, xyz, ws = _case(3)
    r = np.random.default_rng(4)
    gs = r.normal(size=x16.shape[0]).astype(np.float32) * 1e-2
    ga = (r.normal(size=(x16.shape[0], 3)) * 1e-2).astype(np.float16)
    fo = of.field_forward(xyz, ws, x16)
    fb = of.forward_bounds(fo, ws)
    bo = of.field_backward(fo, ws, gs, ga)
    bb = of.backward_bounds(fo, bo, ws, fb)
    # independent autograd of the f32-accumulating emulation
    w = [torch.from_numpy(of.r16(v).astype(np.float32)).requires_grad_(True) for v in ws]
    x = torch.from_numpy(x16.astype(np.float32)).requires_grad_(True)
    ste = lambda t: t + (t.half().float() - t).detach()  # noqa: E731  f16 rounding, identity grad
    a1 = torch.relu(ste(x @ w[0].t() + w[1]))
    a2 = torch.relu(ste(a1 @ w[2].t() + w[3]))
    h = ste(a2 @ w[4].t() + w[5])
    sigma = torch.exp(h[:, 0] + torch.from_numpy(of.gaussian(xyz)))
    alb = torch.sigmoid(h[:, 1:])
    # the f16 rounding of the gradients themselves is applied by hooks
    for t in (h, a1, a2):
        t.register_hook(lambda g: g.half().float())
    loss = (sigma * torch.from_numpy(gs)).sum() + (alb * torch.from_numpy(ga.astype(np.float32))).sum()
    loss.backward()
    dx = x.grad.half().numpy().astype(np.float64)
    dd = np.abs(dx - bo["d_enc"].astype(np.float64))
    # the emulation rounds at slightly different points (the sigmoid grad in
    # f32 before the f16 hook): compare by rel-norm, and against the windows
    rel = np.linalg.norm(dx - bo["d_enc"]) / np.linalg.norm(bo["d_enc"].astype(np.float64))
    assert rel < 2e-3
    assert (dd <= bb["d_enc"] + of.ulp16(bo["d_enc"])).mean() > 0.99
    for i, (a, b, win) in enumerate(zip(w, bo["grads"], bb["grads"])):
        err = np.abs(a.grad.double().numpy() - b)
        assert np.all(err <= win + 2e-3 * np.abs(b).max()), i


def test_bg_forward_matches_f32_emulation():
    r = np.random.default_rng(5)
    d = r.normal(size=(4096, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    lim = lambda k: 1 / np.sqrt(k)  # noqa: E731
    ws = [r.uniform(-lim(39), lim(39), (64, 39)).astype(np.float32),
          r.uniform(-lim(39), lim(39), 64).astype(np.float32),
          r.uniform(-lim(64), lim(64), (3, 64)).astype(np.float32),
          r.uniform(-lim(64), lim(64), 3).astype(np.float32)]
    bo = of.bg_forward(d, ws)
    bb = of.bg_bounds(bo, ws)
    w = [torch.from_numpy(of.r16(v).astype(np.float32)) for v in ws]
    x = torch.from_numpy(bo["x"].astype(np.float32))
    a1 = torch.relu((x @ w[0].t() + w[1]).half().float())
    o = (a1 @ w[2].t() + w[3]).half().float()
    bg = torch.sigmoid(o).half().numpy().astype(np.float64)
    assert np.all(np.abs(bg - bo["bg"]) <= bb["dbg"])
