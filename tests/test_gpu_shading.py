"""GPU tests of the non-albedo train steps (textureless / lambertian shading,
reference nerf/network_grid.py:90-144, nerf/renderer.py:485-494,
nerf/utils.py:346-359): the native step (csrc/shade.hip + the 7 M-row field
launches, nerf/native_step.py)

* against the CPU oracle of the shading math (oracle/field.py shade_forward /
  shade_backward) on the step's own field values: normals to f32 rounding,
  colours bit-exact up to f16 boundary flips, orientation loss, stencil and
  albedo gradients;
* the stencil rows (interleaved: row 7 i = sample i, 7 i + 1 + a = its
  stencil point a) equal clamp(x +- eps e_a, -bound, bound) bit for bit;
* against the autograd shading step (the reference's composition of
  common_forward x 7 + safe_normalize + lambertian + orientation loss, on the
  same kernels) fed the same rays, noise, light and SDS gradient;
* graph-replayed training with the reference's shading schedule runs.
Each under fp16 autocast (the reference's -O) and bf16 autocast (the C5
option: the oracle's precision("bf16"), tolerances scaled to bf16's 8-bit
significand).
"""
import numpy as np
import pytest
import torch

import oracle.field as of

pytestmark = pytest.mark.gpu


DTYPES = [torch.float16, torch.bfloat16]
ULP1 = {torch.float16: 2.0 ** -10, torch.bfloat16: 2.0 ** -7}  # spacing at 1.0


def _trainer(res, seed, graph=False, dtype=torch.float16):
    import bench
    return bench.make_trainer(res, seed, 0, 1, True, graph=graph,
                              bf16=dtype == torch.bfloat16)


def _np(t):
    return t.float().cpu().numpy() if t.dtype == torch.bfloat16 else t.cpu().numpy()


def _native(trainer, data, shading, ratio, seed=11, step=1234):
    from nerf.native_step import NativeAlbedoStep
    res = data.H
    nat = NativeAlbedoStep(trainer, res, res, shading, ratio)
    batch = data.collate([0])
    nat.prologue(batch["pose"], batch["intrinsics"], seed, step)
    nat.body()
    nat.embedding_backward()
    torch.cuda.synchronize()
    return nat, batch


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shading,ratio", [("textureless", 0.1), ("lambertian", 0.1)])
def test_shading_kernels_match_oracle(gpu, shading, ratio, dtype):
    with of.precision("bf16" if dtype == torch.bfloat16 else "f16"):
        _shading_kernels_match_oracle(gpu, shading, ratio, dtype)


def _shading_kernels_match_oracle(gpu, shading, ratio, dtype):
    trainer, data = _trainer(64, 3, dtype=dtype)
    for _ in range(3):
        trainer.train_iteration(data.collate([0]))
    nat, _ = _native(trainer, data, shading, ratio)
    M = int(nat.counter[0])
    assert M > 1000 and int(nat.m7) == 7 * M
    x = nat.xyzs[:M].cpu().numpy()
    x7 = nat.xyz_field[:7 * M].view(M, 7, 3).cpu().numpy()
    np.testing.assert_array_equal(x7[:, 0], x)
    for a in range(6):
        want = x.copy()
        want[:, a // 2] = want[:, a // 2] + np.float32(-1e-2 if a & 1 else 1e-2)
        np.testing.assert_array_equal(x7[:, 1 + a], np.clip(want, -1, 1))
    sig7 = nat.sigma_field[:7 * M].view(M, 7).cpu().numpy()
    np.testing.assert_array_equal(nat.sigma[:M].cpu().numpy(), sig7[:, 0])
    assert nat.albedo.dtype == dtype and nat.color.dtype == dtype
    alb = _np(nat.albedo[:7 * M].view(M, 7, 3)[:, 0])
    dirs = nat.dirs[:M].cpu().numpy()
    light = nat.light.cpu().numpy()
    np.testing.assert_allclose(np.linalg.norm(light), 1.0, rtol=1e-6)
    fo = of.shade_forward(sig7[:, 0], sig7[:, 1:].T, alb, dirs, light, ratio, shading)
    np.testing.assert_allclose(nat.normal[:M].cpu().numpy(), fo["normal"], rtol=2e-6, atol=2e-7)
    col = _np(nat.color[:M])
    flips = (col != fo["color"]).any(1)
    # a colour may take the neighbouring value only where the f32 normal
    # differs in its last bits and the product sits on a rounding boundary
    assert flips.mean() < 1e-3, flips.mean()
    np.testing.assert_allclose(col.astype(np.float32), fo["color"].astype(np.float32),
                               atol=2 * ULP1[dtype], rtol=0)
    want_orient = fo["orient"].astype(np.float64).sum() / of.padded_rows(M)
    np.testing.assert_allclose(float(nat.orient), want_orient, rtol=1e-5)
    # backward, fed the step's own compositing gradient
    scale = float(trainer.scaler._scale) if trainer.scaler.is_enabled() else 1.0
    gsp, ga = of.shade_backward(fo, alb, dirs, _np(nat.grad_color[:M]), scale,
                                trainer.opt.lambda_orient, of.padded_rows(M), ratio, shading)
    g7 = nat.grad_sigma_field[:7 * M].view(M, 7).cpu().numpy()
    np.testing.assert_array_equal(g7[:, 0], nat.grad_sigma[:M].cpu().numpy())
    got = g7[:, 1:].T
    clean = ~flips
    np.testing.assert_allclose(got[:, clean], gsp[:, clean], rtol=1e-4,
                               atol=1e-6 * np.abs(gsp).max())
    ga_got = _np(nat.grad_albedo[:7 * M].view(M, 7, 3))
    assert not ga_got[:, 1:].any()  # stencil rows carry no albedo gradient
    if shading == "lambertian":
        np.testing.assert_allclose(ga_got[:, 0][clean].astype(np.float32),
                                   ga[clean].astype(np.float32), rtol=2 * ULP1[dtype],
                                   atol=1e-7)
    else:
        assert not ga_got[:, 0].any()


def _autograd_grads(trainer, nat, batch, shading, ratio, res, dtype=torch.float16):
    """The autograd shading step on the native step's draws: same rays, march
    noise, light and SDS gradient."""
    model = trainer.model
    trainer.optimizer.zero_grad(set_to_none=True)
    g_img = nat.g_image.view(1, 3, res, res).clone()
    trainer.guidance.sds_grad = lambda text_z, pred_rgb, *a, **k: (pred_rgb, g_img)
    model.march_noises = nat.noises.clone()
    trainer.opt.light_d = nat.light.clone()
    eager = {"H": res, "W": res, "rays_o": nat.rays_o.view(1, -1, 3).clone(),
             "rays_d": nat.rays_d.view(1, -1, 3).clone(), "dir": batch["dir"]}
    try:
        with torch.autocast("cuda", dtype=dtype):
            loss = trainer.train_step(eager, shading, ratio, trainer.text_z[batch["dir"]])[2]
        trainer.backward_only(loss)
    finally:
        del model.march_noises
        del trainer.guidance.sds_grad
        del trainer.opt.light_d
    torch.cuda.synchronize()
    return loss


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shading,ratio", [("textureless", 0.1), ("lambertian", 0.1)])
def test_native_shaded_step_matches_autograd_step(gpu, shading, ratio, dtype):
    res = 64
    trainer, data = _trainer(res, 7, dtype=dtype)
    batch = data.collate([0])
    for _ in range(3):
        trainer.train_iteration(batch)
    params = [p for p in trainer.model.parameters() if p.requires_grad]
    snap = [p.detach().clone() for p in params]
    nat, _ = _native(trainer, data, shading, ratio)
    got = [p.grad.detach().clone() for p in params]
    got_loss = float(nat.loss)
    with torch.no_grad():
        for p, v in zip(params, snap):
            p.copy_(v)
    loss = _autograd_grads(trainer, nat, batch, shading, ratio, res, dtype)
    assert int(trainer.model.last_counter[0]) == int(nat.counter[0])
    np.testing.assert_allclose(float(loss.detach()), got_loss, rtol=1e-5)
    for p, g in zip(params, got):
        assert p.grad is not None
        ref = p.grad.double()
        err = (g.double() - ref).norm() / ref.norm().clamp(min=1e-30)
        # same field kernels; the shading restatement rounds in the same places
        # but its f32 sums may order differently (rare colour flips)
        assert err < 2 * ULP1[dtype], (tuple(p.shape), float(err))


@pytest.mark.parametrize("dtype", DTYPES)
def test_shaded_graph_training_runs(gpu, dtype):
    """The reference's schedule after albedo_iters: 20 % albedo, 40 %
    textureless, 40 % lambertian; every shading graph-replayed natively."""
    trainer, data = _trainer(64, 9, graph=True, dtype=dtype)
    trainer.opt.albedo_iters = 2
    model = trainer.model
    before = [p.detach().clone() for p in model.parameters() if p.requires_grad]
    losses = [float(trainer.train_iteration(data.collate([i % 4]))) for i in range(30)]
    assert all(np.isfinite(losses))
    kinds = {k[0] for k, g in trainer._graphs.items()}
    assert {"textureless", "lambertian"} <= kinds
    assert all(g.native is not None for g in trainer._graphs.values())
    after = [p.detach() for p in model.parameters() if p.requires_grad]
    for a, b in zip(after, before):
        assert torch.isfinite(a).all() and not torch.equal(a, b)


@pytest.mark.parametrize("two_pass", [False, True])
def test_shaded_loss_is_fresh_each_step_without_entropy(gpu, two_pass):
    """lambda_entropy = 0 with a shading: the loss is lambda_orient * orient of
    this step (utils.py:385-402 builds it fresh), not a sum over steps; repeated
    body() calls on the same draws give the same loss."""
    trainer, data = _trainer(64, 5)
    for _ in range(3):  # occupancy refresh: the march emits samples
        trainer.train_iteration(data.collate([0]))
    trainer.opt.lambda_entropy = 0.0
    trainer.fused_backward = not two_pass
    from nerf.native_step import NativeAlbedoStep
    shading = "lambertian" if not two_pass else "albedo"
    nat = NativeAlbedoStep(trainer, 64, 64, shading, 0.1)
    batch = data.collate([0])
    losses = []
    for _ in range(3):
        # the prologue resets the march counter: every body() sees the same draws
        nat.prologue(batch["pose"], batch["intrinsics"], 3, 77)
        losses.append(float(nat.body()))
    torch.cuda.synchronize()
    assert int(nat.counter[0]) > 1000
    assert losses[0] == losses[1] == losses[2], losses
    if shading != "albedo":
        want = trainer.opt.lambda_orient * float(nat.orient)
        np.testing.assert_allclose(losses[0], want, rtol=1e-6)
        assert losses[0] > 0
