"""The product NeRFRenderer.run() (the --cuda_ray-off renderer: coarse uniform
samples + sample_pdf importance samples, reference nerf/renderer.py:15-49,
301-443) on the GPU, against the CPU oracle of the same path
(oracle/cpu_render.py CPUNeRF.run, pure torch f32) with the SAME parameters:
the grid encoder, sigma MLP and background net weights are copied over.

Eval mode (sample_pdf's deterministic u), no perturbation, albedo shading,
fp32 (the reference's C1 configuration has no autocast on CPU).  Both sides are
f32 with different summation orders (GPU grid kernel / hipBLAS GEMMs vs CPU
torch), so the images agree to f32 accumulation noise: 2e-5 abs on colours in
[0, 1].  The march-free path also runs the product FreqEncoder and
near_far_from_aabb kernels."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(gpu, seed=0, emb_scale=0.5):
    import main
    import oracle.cpu_render as cr
    from nerf.network_grid import NeRFNetwork
    opt = main.parse_opt(["--text", "a hamburger", "--h", "32", "--w", "32"])
    assert not opt.cuda_ray and not opt.fp16
    torch.manual_seed(seed)
    net = NeRFNetwork(opt).to(gpu)
    with torch.no_grad():
        net.encoder.embeddings.uniform_(-emb_scale, emb_scale)
    net.eval()
    ref = cr.CPUNeRF(bound=opt.bound, min_near=opt.min_near)
    with torch.no_grad():
        ref.encoder.embeddings.copy_(net.encoder.embeddings.cpu())
        for dst, src in ((ref.sigma_net, net.sigma_net.net), (ref.bg_net, net.bg_net.net)):
            lins = [m for m in dst if isinstance(m, torch.nn.Linear)]
            for a, b in zip(lins, src):
                a.weight.copy_(b.weight.cpu())
                a.bias.copy_(b.bias.cpu())
        ref.aabb = net.aabb_infer.detach().cpu().clone()
    return opt, net, ref


@pytest.mark.parametrize("res", [32, 64])
def test_run_matches_cpu_oracle(gpu, res):
    """64 x 64 is BASELINE configs[0]'s render size (C1)."""
    from nerf.provider import NeRFDataset
    opt, net, ref = _models(gpu)
    data = NeRFDataset(opt, device=gpu, type="test", H=res, W=res, size=8).collate([2])
    rays_o, rays_d = data["rays_o"], data["rays_d"]
    light = torch.tensor([0.0, 0.0, 1.0], device=gpu)
    with torch.no_grad():
        out = net.render(rays_o, rays_d, staged=False, perturb=False, light_d=light,
                         ambient_ratio=1.0, shading="albedo", bg_color=None,
                         num_steps=opt.num_steps, upsample_steps=opt.upsample_steps)
        img_ref, ws_ref = ref.run(rays_o[0].cpu(), rays_d[0].cpu(), opt.num_steps,
                                  opt.upsample_steps, perturb=False, det=True)
    img = out["image"].reshape(-1, 3).cpu()
    ws = out["weights_sum"].reshape(-1).cpu()
    assert torch.isfinite(img).all()
    assert float(ws.max()) > 0.05  # the scene is not empty
    np.testing.assert_allclose(ws.numpy(), ws_ref.numpy(), rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(img.numpy(), img_ref.numpy(), rtol=1e-4, atol=2e-5)


def _ref_grads(ref, rays_o, rays_d, gi, opt):
    img, _ = ref.run(rays_o, rays_d, opt.num_steps, opt.upsample_steps, perturb=False, det=True)
    (img * gi).sum().backward()
    out = [ref.encoder.embeddings.grad.detach().double().clone()]
    for seq in (ref.sigma_net, ref.bg_net):
        for m in seq:
            if isinstance(m, torch.nn.Linear):
                out += [m.weight.grad.detach().double().clone(), m.bias.grad.detach().double().clone()]
    return out


def test_run_train_step_backward_matches_cpu_oracle(gpu):
    """Gradients of run()'s output (albedo, deterministic samples) w.r.t. every
    parameter.  The path's cumprod transmittance (renderer.py:415-418, 1 - alpha
    + 1e-15) makes its backward ill-conditioned where alpha -> 1, so f32 results
    are compared against the oracle run in FLOAT64 and must be as close to it
    as the oracle's own f32 CPU execution (the reference's C1 numerics) is,
    within 3x, and within 1e-2 rel-norm outright."""
    import copy
    from nerf.provider import NeRFDataset
    opt, net, ref = _models(gpu, seed=1, emb_scale=0.2)
    data = NeRFDataset(opt, device=gpu, type="test", H=24, W=24, size=8).collate([1])
    rays_o, rays_d = data["rays_o"], data["rays_d"]
    light = torch.tensor([0.0, 0.0, 1.0], device=gpu)
    g = torch.Generator().manual_seed(3)
    gi = torch.randn(rays_o.shape[1], 3, generator=g)
    out = net.render(rays_o, rays_d, staged=False, perturb=False, light_d=light,
                     ambient_ratio=1.0, shading="albedo", bg_color=None,
                     num_steps=opt.num_steps, upsample_steps=opt.upsample_steps)
    (out["image"].reshape(-1, 3) * gi.to(gpu)).sum().backward()
    got = [net.encoder.embeddings.grad.detach().cpu().double()]
    for seq in (net.sigma_net.net, net.bg_net.net):
        for m in seq:
            got += [m.weight.grad.detach().cpu().double(), m.bias.grad.detach().cpu().double()]
    ref64 = copy.deepcopy(ref).double()
    ref64.aabb = ref.aabb.double()
    exact = _ref_grads(ref64, rays_o[0].cpu().double(), rays_d[0].cpu().double(), gi.double(), opt)
    cpu32 = _ref_grads(ref, rays_o[0].cpu(), rays_d[0].cpu(), gi, opt)
    for a, c, e in zip(got, cpu32, exact):
        n = e.norm().clamp(min=1e-30)
        err_gpu = float((a - e).norm() / n)
        err_cpu = float((c - e).norm() / n)
        print(tuple(e.shape), f"gpu {err_gpu:.2e} cpu-f32 {err_cpu:.2e}")
        assert err_gpu <= 3 * err_cpu + 1e-6 and err_gpu < 1e-2, (tuple(e.shape), err_gpu, err_cpu)
