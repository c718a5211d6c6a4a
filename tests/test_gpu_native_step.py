"""GPU tests of the native albedo train step (nerf/native_step.py, csrc/step.hip):

* the prologue's rays / near-far are bit-identical to dfhip_get_rays and
  near_far_from_aabb (same device code), its draws are deterministic in
  (seed, step), fresh per step, and distributed as the reference's
  (U[0, 1) noise, w(t) * N(0, 1) SDS gradient, t in [min_step, max_step]);
* one native step (prologue -> march -> field -> compositing -> head ->
  entropy -> backward -> binned embedding backward) gives bit-identical
  gradients to the autograd step fed the same rays, noise and SDS gradient;
* graph-replayed native training runs, stays finite and updates every tensor.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(res, seed, graph=False, fused=True):
    import bench
    return bench.make_trainer(res, seed, 0, 1, fused, graph=graph)


def test_prologue_rays_near_far_and_draws(gpu):
    import _dfhip
    import raymarching
    from nerf.native_step import NativeAlbedoStep, eligible
    from nerf.utils import get_rays_host_pose
    trainer, data = _trainer(48, 3)
    assert eligible(trainer, "albedo")
    nat = NativeAlbedoStep(trainer, 48, 48)
    batch = data.collate([0])
    nat.prologue(batch["pose"], batch["intrinsics"], 5, 17)
    want = get_rays_host_pose(batch["pose"], batch["intrinsics"], 48, 48, gpu)
    assert torch.equal(nat.rays_o, want["rays_o"][0]) and torch.equal(nat.rays_d, want["rays_d"][0])
    ne, fa = raymarching.near_far_from_aabb(want["rays_o"][0], want["rays_d"][0],
                                            trainer.model.aabb_train)
    assert torch.equal(nat.nears, ne) and torch.equal(nat.fars, fa)
    assert int(nat.counter.abs().sum()) == 0
    noise1, g1 = nat.noises.clone(), nat.g_image.clone()
    assert 0 <= float(noise1.min()) and float(noise1.max()) < 1
    assert abs(float(noise1.mean()) - 0.5) < 0.03
    # w(t) * eps: one w per step; eps ~ N(0, 1)
    alphas = trainer.guidance.alphas
    w = float(g1.std())
    ws_allowed = 1 - alphas[trainer.guidance.min_step:trainer.guidance.max_step + 1]
    assert float(ws_allowed.min()) * 0.9 < w < float(ws_allowed.max()) * 1.1
    assert abs(float(g1.mean())) < 0.05 * w
    nat.prologue(batch["pose"], batch["intrinsics"], 5, 17)
    assert torch.equal(nat.noises, noise1) and torch.equal(nat.g_image, g1)
    nat.prologue(batch["pose"], batch["intrinsics"], 5, 18)
    assert not torch.equal(nat.noises, noise1)
    nat.prologue(batch["pose"], batch["intrinsics"], 6, 17)
    assert not torch.equal(nat.noises, noise1)
    torch.cuda.synchronize()
    _dfhip.load()


@pytest.mark.parametrize("fused", [True, False])
def test_native_step_matches_autograd_step(gpu, fused):
    """fused: one backward of SDS + scaled loss; not fused: the reference's two
    passes (sd.py:115 then utils.py:708), gradients accumulated."""
    from nerf.native_step import NativeAlbedoStep
    res = 64
    trainer, data = _trainer(res, 7, fused=fused)
    batch = data.collate([0])
    for _ in range(3):  # density-grid refresh + a few eager steps
        trainer.train_iteration(batch)
    model = trainer.model
    params = [p for p in model.parameters() if p.requires_grad]
    snap = [p.detach().clone() for p in params]

    nat = NativeAlbedoStep(trainer, res, res)
    nat.prologue(batch["pose"], batch["intrinsics"], 11, 1234)
    nat.body()
    nat.embedding_backward()
    torch.cuda.synchronize()
    got = [p.grad.detach().clone() for p in params]
    got_count = nat.counter.clone()
    got_loss = nat.loss.clone()
    got_rgb = nat.out_image.clone()  # pred_rgb, channel-major [3, N]
    assert int(got_count[0]) > 0

    # the autograd step on the same inputs
    with torch.no_grad():
        for p, v in zip(params, snap):
            p.copy_(v)
    trainer.optimizer.zero_grad(set_to_none=True)
    g_img = nat.g_image.view(1, 3, res, res).clone()
    trainer.guidance.sds_grad = lambda text_z, pred_rgb, *a, **k: (pred_rgb, g_img)
    model.march_noises = nat.noises.clone()
    model.device_count_march = True
    eager = {"H": res, "W": res, "rays_o": nat.rays_o.view(1, -1, 3).clone(),
             "rays_d": nat.rays_d.view(1, -1, 3).clone(), "dir": batch["dir"]}
    text_z = trainer.text_z[batch["dir"]]
    try:
        with torch.autocast("cuda", dtype=torch.float16):
            pred_rgb, _, loss = trainer.train_step(eager, "albedo", 1.0, text_z)
        trainer.backward_only(loss)
    finally:
        model.device_count_march = False
        del model.march_noises
        del trainer.guidance.sds_grad
    torch.cuda.synchronize()
    assert torch.equal(model.last_counter, got_count)
    assert torch.equal(loss.detach().float(), got_loss)
    # the forward's output (with fused: from the head's combined launch)
    assert torch.equal(pred_rgb.detach().float().reshape(-1), got_rgb.reshape(-1))
    for p, g in zip(params, got):
        assert p.grad is not None
        assert torch.equal(p.grad, g), (tuple(p.shape), float((p.grad - g).abs().max()))


@pytest.mark.parametrize("fused", [True, False])
def test_native_graph_training_runs(gpu, fused):
    trainer, data = _trainer(64, 9, graph=True, fused=fused)
    model = trainer.model
    before = [p.detach().clone() for p in model.parameters() if p.requires_grad]
    losses = []
    for i in range(40):
        loss = trainer.train_iteration(data.collate([i % 4]))
        losses.append(float(loss))
    assert len(trainer._graphs) == 1
    g = next(iter(trainer._graphs.values()))
    assert g.native is not None
    assert all(np.isfinite(losses))
    assert model.mean_density > 0
    assert int(model.step_counter[:, 0].min()) > 0
    after = [p.detach() for p in model.parameters() if p.requires_grad]
    for a, b in zip(after, before):
        assert torch.isfinite(a).all()
        assert not torch.equal(a, b)


def test_checkpoint_round_trip_resumes(gpu, tmp_path):
    """Trainer.save_checkpoint / load_checkpoint (reference utils.py:847-968)
    after graph-replayed native steps: the reference's keys (model incl. the
    occupancy state, mean_count / mean_density, optimizer, scaler, scheduler)
    round-trip exactly into a fresh trainer, which then keeps training."""
    trainer, data = _trainer(64, 21, graph=True)
    for i in range(20):
        trainer.train_iteration(data.collate([i % 4]))
    torch.cuda.synchronize()
    trainer.ckpt_path = str(tmp_path)
    trainer.save_checkpoint("ck", full=True)
    ck = torch.load(tmp_path / "ck.pth", map_location=gpu, weights_only=True)
    for key in ("epoch", "global_step", "stats", "mean_count", "mean_density", "optimizer",
                "lr_scheduler", "scaler", "model"):
        assert key in ck, key
    for key in ("encoder.embeddings", "sigma_net.net.0.weight", "density_grid",
                "density_bitfield", "step_counter", "aabb_train"):
        assert key in ck["model"], key
    assert ck["global_step"] == trainer.global_step == 20

    fresh, _ = _trainer(64, 22, graph=True)
    fresh.ckpt_path = str(tmp_path)
    fresh.load_checkpoint(str(tmp_path / "ck.pth"))
    want, got = trainer.model.state_dict(), fresh.model.state_dict()
    assert want.keys() == got.keys()
    for k in want:
        assert torch.equal(want[k], got[k]), k
    assert fresh.global_step == 20
    assert int(fresh.model.mean_count) == int(trainer.model.mean_count)
    assert float(fresh.model.mean_density) == float(trainer.model.mean_density)
    assert float(fresh.scaler.get_scale()) == float(trainer.scaler.get_scale())
    so, sf = trainer.optimizer.state_dict()["state"], fresh.optimizer.state_dict()["state"]
    assert so.keys() == sf.keys()
    for i in so:
        for name in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(so[i][name].to(gpu), sf[i][name].to(gpu)), (i, name)
    losses = [float(fresh.train_iteration(data.collate([i % 4]))) for i in range(5)]
    assert all(np.isfinite(losses))
    assert fresh.global_step == 25


def test_optimizer_in_graph_matches_host_lr_adam(gpu):
    """Single GPU: the native step's graph ends with GradScaler + Adam reading
    device learning rates the prologue writes (dfhip_adam_amp_step_lr_dev).
    Over 20 steps of LambdaLR-decayed rates (main.py:131), crossing a density
    refresh, the parameters, Adam moments, step counts and the loss scale equal
    a twin trainer whose steps run the same launches eagerly and the optimizer
    as the host-lr NativeAdamAmp.step() (nerf/optim.py), bit for bit."""
    # one trainer after the other: make_trainer reseeds the global RNGs the
    # camera sampler and the density refresh draw from, so both see the same
    # poses and jitter
    def run(hook):
        tr, dt = _trainer(64, 5, graph=True)
        tr.opt.iters = 50  # decay fast enough that every step's lr differs in f32
        tr.step_hook = hook
        for i in range(20):
            tr.train_iteration(dt.collate([i % 4]))
        torch.cuda.synchronize()
        return tr

    def host_optimizer(g):
        g.optimizer_in_graph = False  # optimizer_step() then runs the host-lr Adam
        g.native.body()
        g.native.embedding_backward()
        for p, gr in g.grads:
            p.grad = gr
    a = run(None)
    b = run(host_optimizer)
    torch.cuda.synchronize()
    ga = next(iter(a._graphs.values()))
    assert ga.native is not None and ga.optimizer_in_graph
    lrs = [g["lr"] for g in a.optimizer.param_groups]
    assert lrs == [g["lr"] for g in b.optimizer.param_groups]
    assert lrs[0] < a.optimizer.param_groups[0]["initial_lr"]  # the schedule moved
    for pa, pb in zip(a.model.parameters(), b.model.parameters()):
        assert torch.equal(pa, pb)
    sa, sb = a.optimizer.state_dict()["state"], b.optimizer.state_dict()["state"]
    for i in sa:
        for name in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[i][name], sb[i][name]), (i, name)
    assert float(a.scaler.get_scale()) == float(b.scaler.get_scale())


def test_eval_frame_operands_follow_graph_training(gpu):
    """The fused eval renderer caches its launch operands (f32 weights, f16
    table, corner quads) between frames.  The graph-replayed step updates the
    parameters in place with the native Adam (no torch version bump), so a
    render -> train -> render sequence (the reference's periodic eval,
    utils.py train() -> evaluate_one_epoch) must see the new parameters: the
    second frame equals a frame rendered with the cache dropped."""
    from scenes import camera_rays
    trainer, data = _trainer(64, 13, graph=True)
    m = trainer.model
    for i in range(3):
        trainer.train_iteration(data.collate([i % 4]))
    o, d = camera_rays(32, 32, 13, radius=1.6)
    rays_o = torch.from_numpy(o).to(gpu)[None]
    rays_d = torch.from_numpy(d).to(gpu)[None]

    def frame():
        m.eval()
        try:
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
                out = m.render(rays_o, rays_d, staged=True, perturb=False, light_d=None,
                               ambient_ratio=1.0, shading="albedo", force_all_rays=True,
                               bg_color=None, **vars(trainer.opt))
        finally:
            m.train()
        torch.cuda.synchronize()
        return out["image"].float().clone()

    a = frame()
    assert m.__dict__.get("_infer_operands") is not None  # the fused path ran and cached
    for i in range(3):
        trainer.train_iteration(data.collate([(i + 3) % 4]))
    g = next(iter(trainer._graphs.values()))
    assert g.native is not None and g.optimizer_in_graph
    b = frame()
    m.__dict__.pop("_infer_operands", None)
    c = frame()
    assert torch.equal(b, c)
    assert not torch.equal(a, b)  # training moved the field
