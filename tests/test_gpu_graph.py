"""GPU tests of the host-sync-free train step (nerf/graph.py):

* march_rays_train_dev emits exactly march_rays_train's samples (bit-exact on
  the live rows, same ray table and count) without a host sync;
* the mixed-precision compositing (f16 colours read and their gradient written
  as f16) equals the reference's f32 compositing of the upcast colours, with
  the f32 colour gradient rounded to f16 once;
* one HIP-graph replay of the step gives the gradients of the same step run
  eagerly from the same RNG state (the deferred embedding backward included);
* a graph-replay training run (crossing density-grid refreshes) stays finite
  and updates every trainable tensor.
"""
import numpy as np
import pytest
import torch

from scenes import march_inputs

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def test_march_dev_matches_march(gpu):
    import raymarching
    rays_o, rays_d, nears, fars, _, bf = march_inputs(96, 96, seed=3)
    args = [_t(rays_o, gpu), _t(rays_d, gpu), 1.0, _t(bf, gpu), 1, 128, _t(nears, gpu),
            _t(fars, gpu)]
    c0 = torch.zeros(2, dtype=torch.int32, device=gpu)
    torch.manual_seed(11)
    x0, d0, l0, r0 = raymarching.march_rays_train(*args, c0, -1, True, 128, True, 0.0, 512)
    c1 = torch.zeros(2, dtype=torch.int32, device=gpu)
    torch.manual_seed(11)
    x1, d1, l1, r1 = raymarching.march_rays_train_dev(*args, c1, True, 0.0, 512)
    m = int(c1[0])
    assert torch.equal(c0, c1) and m > 0
    assert x1.shape[0] == rays_o.shape[0] * 512
    assert torch.equal(raymarching.live_rows(x1), c1[:1])
    assert torch.equal(r0, r1)
    assert torch.equal(x0[:m], x1[:m]) and torch.equal(d0[:m], d1[:m])
    assert torch.equal(l0[:m], l1[:m])


def test_composite_mixed_matches_f32(gpu):
    import raymarching
    rays_o, rays_d, nears, fars, _, bf = march_inputs(64, 64, seed=4)
    c = torch.zeros(2, dtype=torch.int32, device=gpu)
    x, d, deltas, rays = raymarching.march_rays_train_dev(
        _t(rays_o, gpu), _t(rays_d, gpu), 1.0, _t(bf, gpu), 1, 128, _t(nears, gpu),
        _t(fars, gpu), c, True, 0.0, 512)
    m = int(c[0])
    g = torch.Generator(device=gpu).manual_seed(0)
    sig = torch.rand(x.shape[0], device=gpu, generator=g) * 30
    rgb16 = torch.rand(x.shape[0], 3, device=gpu, generator=g).half()
    gws = torch.randn(rays.shape[0], device=gpu, generator=g)
    gimg = torch.randn(rays.shape[0], 3, device=gpu, generator=g)

    # mixed path (autocast, f16 colours, capacity rows)
    s1 = sig.clone().requires_grad_()
    c1 = rgb16.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.float16):
        ws1, dp1, im1 = raymarching.composite_rays_train(s1, c1, deltas, rays, 1e-4)
    torch.autograd.backward([ws1, im1], [gws, gimg])
    assert c1.grad.dtype == torch.float16

    # reference form: f32 colours of the live rows, gradient cast to f16 after
    s2 = sig[:m].clone().requires_grad_()
    c2 = rgb16[:m].float().requires_grad_()
    r2 = rays.clone()  # no live-rows attribute: plain dense path
    ws2, dp2, im2 = raymarching.composite_rays_train(s2, c2, deltas[:m].clone(), r2, 1e-4)
    torch.autograd.backward([ws2, im2], [gws, gimg])
    assert torch.equal(ws1, ws2) and torch.equal(dp1, dp2) and torch.equal(im1, im2)
    assert torch.equal(s1.grad[:m], s2.grad)
    assert torch.equal(c1.grad[:m], c2.grad.half())


def _snapshot(model):
    return [p.detach().clone() for p in model.parameters()]


def _restore(model, snap):
    with torch.no_grad():
        for p, v in zip(model.parameters(), snap):
            p.copy_(v)


def test_graph_step_matches_eager_step(gpu):
    import bench
    from nerf.graph import GraphedTrainStep
    trainer, data = bench.make_trainer(64, 7, 0, 1, True, graph=False)
    batch = data.collate([0])
    for _ in range(3):  # density-grid refresh + a few eager steps
        trainer.train_iteration(batch)
    model = trainer.model
    params = [p for p in model.parameters() if p.requires_grad]
    text_z = trainer.text_z[batch["dir"]]
    snap = _snapshot(model)

    # eager, device-count march, same sequence of RNG draws as the graph
    trainer.optimizer.zero_grad()
    model.device_count_march = True
    torch.cuda.manual_seed(1234)
    with torch.autocast("cuda", dtype=torch.float16):
        loss = trainer.train_step(batch, "albedo", 1.0, text_z)[2]
    trainer.backward_only(loss)
    model.device_count_march = False
    # drop the eager step's autograd graph: its AccumulateGrad nodes are bound
    # to the default stream and would be reused by the capture
    del loss
    want = [p.grad.detach().clone() for p in params]
    want_count = model.last_counter.clone()

    _restore(model, snap)
    stream = torch.cuda.Stream()
    g = GraphedTrainStep(trainer, batch, "albedo", 1.0, text_z, stream, allow_native=False)
    torch.cuda.current_stream().synchronize()
    g.capture()
    torch.cuda.manual_seed(1234)
    g.load(batch, text_z)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(g.counter, want_count)
    for p, w in zip(params, want):
        assert p.grad is not None and p.grad.shape == w.shape
        # upsample / pooling backwards of the SDS stand-in use float atomics
        scale = w.abs().max().clamp(min=1e-12)
        torch.testing.assert_close(p.grad, w, rtol=1e-3, atol=1e-4 * scale)


def test_graph_training_runs(gpu):
    import bench
    trainer, data = bench.make_trainer(64, 9, 0, 1, True, graph=True)
    model = trainer.model
    before = [p.detach().clone() for p in model.parameters() if p.requires_grad]
    losses = []
    for i in range(40):
        loss = trainer.train_iteration(data.collate([i % 4]))
        losses.append(float(loss))
    assert len(trainer._graphs) == 1
    assert all(np.isfinite(losses))
    assert model.mean_density > 0
    assert int(model.step_counter[:, 0].min()) > 0  # every row written by the replays
    after = [p.detach() for p in model.parameters() if p.requires_grad]
    for a, b in zip(after, before):
        assert torch.isfinite(a).all()
        assert not torch.equal(a, b)
