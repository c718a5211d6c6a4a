"""Native GradScaler + Adam step (csrc/optim.hip, nerf/optim.py) against
torch's GradScaler.step / update with a fused torch.optim.Adam on the same
parameters and gradients: same parameters, moments, step counts and scale
(f32 tolerance: torch's kernel is compiled with FMA contraction, ours is not),
including a skipped non-finite step and a scale growth."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(gpu, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    shapes = [(1000, 2), (64, 32), (64,), (4, 64), (4,), (3, 64)]
    ps = [torch.randn(s, device=gpu, generator=g).requires_grad_() for s in shapes]
    groups = [{"params": ps[:1], "lr": 1e-2}, {"params": ps[1:], "lr": 1e-3}]
    opt = torch.optim.Adam(groups, betas=(0.9, 0.99), eps=1e-15, fused=True)
    sc = torch.amp.GradScaler("cuda", init_scale=1024.0, growth_interval=3)
    return ps, opt, sc, g


def test_native_adam_amp_matches_torch(gpu):
    from nerf.optim import NativeAdamAmp, eligible
    pa, oa, sa, g = _setup(gpu, 0)
    pb, ob, sb, _ = _setup(gpu, 0)
    assert eligible(ob, sb)
    nat = NativeAdamAmp(ob, sb)
    for it in range(8):
        grads = [torch.randn(p.shape, device=gpu, generator=g) * 100 for p in pa]
        if it == 4:
            grads[2][3] = float("inf")
        for (p, q, gr) in zip(pa, pb, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        sa.scale(torch.ones((), device=gpu))  # lazy scale init, as backward would
        sb.scale(torch.ones((), device=gpu))
        sa.step(oa)
        sa.update()
        nat.step()
        torch.cuda.synchronize()
        assert float(sa._scale) == float(sb._scale), it
        assert int(sa._growth_tracker) == int(sb._growth_tracker), it
        for p, q in zip(pa, pb):
            torch.testing.assert_close(q, p, rtol=2e-6, atol=1e-7)
            st_a, st_b = oa.state[p], ob.state[q]
            assert float(st_a["step"]) == float(st_b["step"])
            sc = float(st_a["exp_avg"].abs().max())
            torch.testing.assert_close(st_b["exp_avg"], st_a["exp_avg"], rtol=2e-6, atol=1e-6 * sc)
            sq = float(st_a["exp_avg_sq"].abs().max())
            torch.testing.assert_close(st_b["exp_avg_sq"], st_a["exp_avg_sq"], rtol=2e-6,
                                       atol=1e-6 * sq)
    # the inf step was skipped (7 updates) and the scale backed off then grew
    assert float(oa.state[pa[0]]["step"]) == 7.0

