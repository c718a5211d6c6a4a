"""GPU tests of the network / renderer / trainer layers built on the kernels.

The MLP with split-K weight gradients is compared against the plain
nn.Linear/ReLU stack under autocast (torch fp16/fp32 reference of the same op).
The fused single backward and the reference's two-pass backward are each
pinned against the oracle's restatement of their own structure in
tests/test_gpu_step_structures.py.
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def test_mlp_split_k_matches_oracle(gpu):
    """nerf/mlp.py (torch GEMMs + split-K weight gradients, the unfused MLP)
    against the f16-autocast oracle (oracle/field.py mlp_forward): outputs
    inside the order-free rounding windows, weight/bias gradients against the
    exact float64 sums of the f16 graph (2e-5 of the |term| sums + one f16
    ulp of rounding of each upstream activation's window)."""
    import oracle.field as of
    from nerf.mlp import mlp_forward
    torch.manual_seed(0)
    layers = nn.ModuleList([nn.Linear(32, 64), nn.Linear(64, 64), nn.Linear(64, 4)]).to(gpu)
    x = torch.randn(100_003, 32, device=gpu)
    g = torch.randn(100_003, 4, device=gpu) * 1e-2
    with torch.autocast("cuda", dtype=torch.float16):
        y = mlp_forward(x, layers)
    assert y.dtype == torch.float16
    (y.float() * g).sum().backward()
    ws = [p.detach().cpu().numpy() for p in layers.parameters()]
    x16 = x.cpu().numpy().astype(np.float16)
    outs, wins = of.mlp_forward(x16, ws)
    diff = np.abs(y.detach().cpu().numpy().astype(np.float64) - outs[-1].astype(np.float64))
    assert np.all(diff <= wins[-1]), (diff - wins[-1]).max()
    print(f"\noutputs differing from the exact rounding: {(diff > 0).mean():.2e}")
    # gradients of the f16 graph, exact sums
    w16 = [of.r16(w).astype(np.float64) for w in ws[0::2]]
    dy = of.r16(g.cpu().numpy()).astype(np.float64)  # autocast: f16 grad of the f16 output
    acts = [x16.astype(np.float64)] + [o.astype(np.float64) for o in outs[:-1]]
    want, d = [None] * 6, dy
    for i in reversed(range(3)):
        want[2 * i], want[2 * i + 1] = d.T @ acts[i], d.sum(0)
        if i:
            d = np.where(acts[i] > 0, of.r16(d @ w16[i]).astype(np.float64), 0.0)
    for i, (p, w) in enumerate(zip(layers.parameters(), want)):
        got = p.grad.detach().cpu().numpy().astype(np.float64)
        scale = np.abs(w).max()
        # upstream activation windows and flipped ReLU masks move a few terms
        err = np.abs(got - w).max() / scale
        assert p.grad.dtype == torch.float32 and err <= 2e-3, (i, err)


def _trainer(gpu, fused, seed=0):
    import bench
    trainer, data = bench.make_trainer(64, seed, 0, 1, fused)
    return trainer, data


def test_train_iterations_run(gpu):
    trainer, data = _trainer(gpu, True, seed=1)
    before = [p.detach().clone() for p in trainer.model.parameters() if p.requires_grad]
    losses = []
    for _ in range(20):
        loss = trainer.train_iteration(data.collate([0]))
        losses.append(float(loss))
    assert all(np.isfinite(losses))
    m = trainer.model
    assert m.mean_density > 0
    assert int(m.density_bitfield.count_nonzero()) > 0
    for p in m.parameters():
        assert torch.isfinite(p).all()
    # every trainable tensor (encoder, sigma_net, bg_net) was updated by Adam
    after = [p.detach() for p in m.parameters() if p.requires_grad]
    assert len(after) == len(before) and len(after) >= 8
    for a, b in zip(after, before):
        assert not torch.equal(a, b)


def test_inference_render(gpu):
    """Eval branch of run_cuda (alive-ray loop) renders a finite image."""
    trainer, data = _trainer(gpu, True, seed=2)
    trainer.train_iteration(data.collate([0]))
    m = trainer.model
    m.eval()
    from nerf.provider import NeRFDataset
    ds = NeRFDataset(trainer.opt, device=gpu, type="test", H=96, W=96, size=10)
    img, depth = trainer.test_step(ds.collate([3]))
    assert img.shape == (1, 96, 96, 3) and torch.isfinite(img).all()
    assert (img >= 0).all() and (img <= 1.0001).all()


def test_update_extra_state_matches_manual(gpu):
    """Density-grid refresh: EMA-max, mean, packbits threshold (renderer.py:562-615)."""
    import raymarching
    trainer, _ = _trainer(gpu, True, seed=3)
    m = trainer.model
    torch.manual_seed(0)
    m.update_extra_state()
    grid1 = m.density_grid.clone()
    thresh = min(m.mean_density, m.density_thresh)
    want = raymarching.packbits(grid1, thresh)
    assert torch.equal(m.density_bitfield, want)
    assert abs(m.mean_density - float(grid1[grid1 >= 0].mean())) < 1e-5 * max(1.0, m.mean_density)
    # second refresh: EMA-max with decay 0.95
    torch.manual_seed(1)
    m.update_extra_state()
    assert torch.all(m.density_grid >= grid1 * 0.95 - 1e-6)


def test_native_grid_update_matches_torch(gpu):
    """The sync-free refresh (csrc/occupancy.hip) against the reference's torch
    ops on the same state and the same jitter draws."""
    trainer, data = _trainer(gpu, True, seed=4)
    trainer.train_iteration(data.collate([0]))
    trainer.train_iteration(data.collate([1]))
    m = trainer.model
    state = (m.density_grid.clone(), m.density_bitfield.clone(), m.local_step,
             m.step_counter.clone())
    out = {}
    for native in (False, True):
        m.density_grid.copy_(state[0])
        m.density_bitfield.copy_(state[1])
        m.local_step = state[2]
        m.native_grid_update = native
        m.grid_generator = None  # jitter from the default generator, reseeded below
        torch.manual_seed(123)
        with torch.autocast("cuda", dtype=torch.float16):
            m.update_extra_state()
        out[native] = (m.density_grid.clone(), m.density_bitfield.clone(), m.mean_density,
                       m.mean_count)
    g0, b0, md0, mc0 = out[False]
    g1, b1, md1, mc1 = out[True]
    assert torch.equal(g0, g1)
    assert abs(md0 - md1) <= 1e-5 * max(1.0, abs(md0))
    assert mc0 == mc1
    diff = int((b0 != b1).sum())
    # only cells within rounding of the threshold may flip
    assert diff == 0 or diff <= 2


@pytest.mark.parametrize("bg_radius", [1.4, 0.0])
def test_native_ray_head_matches_torch(gpu, bg_radius):
    """Native background mix / depth / mask / entropy (csrc/head.hip) against
    the reference's torch expressions on the same render: outputs and the
    gradients of the background MLP, the colour and the weights."""
    import random
    outs = {}
    for native in (False, True):
        trainer, data = _trainer(gpu, True, seed=5)
        m = trainer.model
        m.native_head = native
        trainer.native_losses = native
        if bg_radius == 0:
            m.bg_radius = 0.0
        torch.manual_seed(7)
        random.seed(7)
        batch = data.collate([0])
        m.update_extra_state()
        trainer.optimizer.zero_grad()
        torch.manual_seed(8)
        with torch.autocast("cuda", dtype=torch.float16):
            pred_rgb, pred_ws, loss = trainer.train_step(batch, "albedo", 1.0)
        g = torch.randn(pred_rgb.shape, device=gpu, generator=torch.Generator(gpu).manual_seed(1))
        trainer._pending_sds = None
        torch.autograd.backward([pred_rgb, loss], [g, None])
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()
                 if p.grad is not None}
        outs[native] = (pred_rgb.detach().clone(), pred_ws.detach().clone(),
                        loss.detach().clone(), grads)
    (r0, w0, l0, g0), (r1, w1, l1, g1) = outs[False], outs[True]
    assert torch.equal(w0, w1)
    torch.testing.assert_close(r1, r0, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-9)
    assert g0.keys() == g1.keys()
    for n in g0:
        scale = g0[n].abs().max().clamp(min=1e-12)
        torch.testing.assert_close(g1[n], g0[n], rtol=2e-2, atol=2e-2 * scale, msg=n)
