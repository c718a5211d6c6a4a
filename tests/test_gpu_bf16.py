"""GPU tests of the bf16 field path (BASELINE configs[4] / C5: bf16 autocast;
the reference has fp16 only, so the oracle is oracle/field.py's bf16
restatement, pinned on CPU against torch's own bf16 autocast in
tests/test_oracle_field_bf16.py).

* march -> dfhip_grid_field_forward_bf16 -> compositing (bf16 colours) ->
  compositing backward -> dfhip_grid_field_backward_bf16 -> binned embedding
  backward (bf16 feature gradients), every stage through the C-ABI, against
  the oracle chain: features bit-exact; sigma / albedo / feature gradients
  inside the propagated bf16 rounding windows (bit-exact where closed);
  compositing 1e-4 rel; weight gradients inside their windows; embedding
  gradients 1e-5 rel-norm against the exact f64 sum of the same bf16 feature
  gradients (f64 accumulation, one f32 rounding per partial image);
* the native bf16 train step gives bit-identical gradients to the autograd
  step under bf16 autocast (same kernels through nerf/field.py), and
  graph-replayed bf16 training at the C5 resolution (256 x 256) runs finite.
Reference: nerf/network_grid.py:13-32,69-87; raymarching.cu:500-693;
gridencoder.cu:226-313.
"""
import numpy as np
import pytest
import torch

import oracle
import oracle.field as of
from test_gpu_field_oracle import MFMA_ULPS, _march, _setup, _unperm

pytestmark = pytest.mark.gpu


def _bf16_np(t):
    return t.float().cpu().numpy()


@pytest.mark.parametrize("seed,emb_scale", [(0, 0.5), (1, 1e-4)])
def test_field_chain_bf16_matches_oracle(gpu, seed, emb_scale):
    import _fieldmlp
    import _gridencoder
    import _raymarching
    enc_mod, layers = _setup(gpu, seed, emb_scale)
    xyzs, deltas, rays, M = _march(gpu, 128, seed)
    N = rays.shape[0]
    assert M > 100_000
    S = float(np.log2(enc_mod.per_level_scale))
    Hb = int(enc_mod.base_resolution)
    gt = enc_mod.gridtype_id
    table = enc_mod.embeddings.detach().bfloat16().contiguous()
    offsets = enc_mod.offsets
    ws = [p.detach().float().contiguous() for lin in layers for p in (lin.weight, lin.bias)]
    ws_np = [w.cpu().numpy() for w in ws]

    enc = torch.empty(M, 32, device=gpu, dtype=torch.bfloat16)
    sigma = torch.empty(M, device=gpu)
    albedo = torch.empty(M, 3, device=gpu, dtype=torch.bfloat16)
    _fieldmlp.grid_field_forward(xyzs, 1.0, table, offsets, S, Hb, gt, False, ws, enc, sigma,
                                 albedo, None)
    x_np = xyzs.cpu().numpy()
    want_enc = of.encode_bf16(x_np, 1.0, enc_mod.embeddings.detach().cpu().numpy(),
                              offsets.cpu().numpy(), S, Hb)
    got_enc = _unperm(_bf16_np(enc))
    assert np.array_equal(got_enc, want_enc), "bf16 features differ"

    with of.precision("bf16"):
        fo = of.field_forward(x_np, ws_np, want_enc)
        fb = of.forward_bounds(fo, ws_np, acc_ulps=MFMA_ULPS)
    s_g, a_g = sigma.cpu().numpy(), _bf16_np(albedo)
    dlog = np.abs(np.log(s_g.astype(np.float64)) - np.log(fo["sigma"].astype(np.float64)))
    assert np.all(dlog <= fb["dlog_sigma"]), \
        f"sigma outside its window: worst excess {(dlog - fb['dlog_sigma']).max():.3e}"
    da = np.abs(a_g.astype(np.float64) - fo["albedo"].astype(np.float64))
    assert np.all(da <= fb["dalbedo"]), \
        f"albedo outside its window: worst excess {(da - fb['dalbedo']).max():.3e}"
    closed = (fb["dh"] == 0).all(1)
    assert np.array_equal(a_g[closed], fo["albedo"][closed])
    print(f"\nM={M}: h windows closed on {closed.mean():.3f} of samples, albedo differs on "
          f"{(a_g != fo['albedo']).any(1).mean():.2e}")

    # compositing with bf16 colours (native mixed form) vs oracle.c on the same inputs
    wsum = torch.empty(N, device=gpu)
    depth = torch.empty(N, device=gpu)
    image = torch.empty(N, 3, device=gpu)
    _raymarching.composite_rays_train_forward_mixed(sigma, albedo, deltas, rays, M, N, 1e-4, wsum,
                                                    depth, image)
    d_np, r_np = deltas.cpu().numpy(), rays.cpu().numpy()
    ow, od, oi = oracle.composite_rays_train_forward(s_g, a_g, d_np, r_np)
    np.testing.assert_allclose(image.cpu().numpy(), oi, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(wsum.cpu().numpy(), ow, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(depth.cpu().numpy(), od, rtol=1e-4, atol=1e-5)

    g = torch.Generator(device="cpu").manual_seed(seed + 10)
    g_img = (torch.randn(N, 3, generator=g) * 1e-2).to(gpu)
    g_ws = (torch.randn(N, generator=g) * 1e-2).to(gpu)
    gs = torch.empty(M, device=gpu)
    grgb = torch.empty(M, 3, device=gpu, dtype=torch.bfloat16)
    _raymarching.composite_rays_train_backward_mixed(g_ws, g_img, sigma, albedo, deltas, rays,
                                                     wsum, image, M, N, 1e-4, gs, grgb)
    ogs, ogc = oracle.composite_rays_train_backward(
        g_ws.cpu().numpy(), g_img.cpu().numpy(), s_g, a_g, d_np, r_np, wsum.cpu().numpy(),
        image.cpu().numpy())
    np.testing.assert_allclose(gs.cpu().numpy(), ogs, rtol=1e-4, atol=1e-7)
    # colour gradients: the f32 product rounded to bf16 once
    gc = _bf16_np(grgb)
    # (round to nearest: half a bf16 ulp, <= 2^-8 relative, plus the 1e-4 of
    # the f32 compositing against the oracle)
    assert np.all(np.abs(gc - ogc) <= (2.0 ** -8 + 2e-4) * np.abs(ogc) + 1e-30)

    d_enc = torch.empty(16, M, 2, device=gpu, dtype=torch.bfloat16)
    partial = torch.empty(_fieldmlp.backward_parts(M) * _fieldmlp.params_count(), device=gpu)
    grads = [torch.empty_like(w) for w in ws]
    _fieldmlp.grid_field_backward(enc, xyzs, 1.0, ws, gs, grgb, d_enc, partial, grads, offsets,
                                  0, S, Hb, gt, False, None, None, 1, None)
    with of.precision("bf16"):
        bo = of.field_backward(fo, ws_np, gs.cpu().numpy(), gc)
        bb = of.backward_bounds(fo, bo, ws_np, fb, acc_ulps=None)
    d_want = bo["d_enc"]
    d_got = _bf16_np(d_enc).transpose(1, 0, 2).reshape(M, 32)
    dd = np.abs(d_got.astype(np.float64) - d_want.astype(np.float64))
    assert np.all(dd <= bb["d_enc"]), \
        f"feature grads outside their window: worst excess {(dd - bb['d_enc']).max():.3e}"
    rel = np.linalg.norm(d_got.astype(np.float64) - d_want) / np.linalg.norm(d_want)
    print(f"feature grads: differing {(dd > 0).mean():.2e}, rel-norm {rel:.2e}")
    assert rel <= 1e-2, rel
    for i, (a, b, w) in enumerate(zip(grads, bo["grads"], bb["grads"])):
        a = a.cpu().numpy().astype(np.float64).reshape(b.shape)
        err = np.abs(a - b)
        assert np.all(err <= w), f"param {i}: worst excess {(err - w).max():.3e}"

    # embedding gradient from the GPU's bf16 feature gradients (binned walk)
    rows = int(offsets[-1].item())
    grad_emb = torch.empty(rows, 2, device=gpu)
    ne, nc, npf = _gridencoder.grid_backward_binned_scratch(M, enc_mod.offsets_host, 16, 2)
    scratch = (torch.empty(ne, device=gpu, dtype=torch.int32),
               torch.empty(nc, device=gpu, dtype=torch.int32), torch.empty(npf, device=gpu))
    launch = _gridencoder.binned_launcher(d_enc, xyzs, 1.0, offsets, enc_mod.offsets_host,
                                          grad_emb, M, None, 3, 2, 16, S, Hb, gt, False, *scratch)
    launch()
    x01 = ((x_np + np.float32(1)) / np.float32(2)).astype(np.float32)
    bits = d_enc.view(torch.int16).cpu().numpy().view(np.uint16)
    e_want = oracle.grid_encode_backward(bits, x01, offsets.cpu().numpy(), 2, S, Hb, blc=False,
                                         bf16=True)
    e_got = grad_emb.cpu().numpy().astype(np.float64)
    rel = np.linalg.norm(e_got - e_want) / max(np.linalg.norm(e_want), 1e-30)
    assert rel <= 1e-5, f"embedding grads rel-norm {rel:.3e}"


def test_native_bf16_step_matches_autograd_step(gpu):
    import bench
    from nerf.native_step import NativeAlbedoStep, eligible
    res = 64
    trainer, data = bench.make_trainer(res, 7, 0, 1, True, bf16=True)
    assert trainer.bf16 and not trainer.scaler.is_enabled()
    # every shading has a native bf16 step (the shaded ones: tests/test_gpu_shading.py)
    assert all(eligible(trainer, s) for s in ("albedo", "textureless", "lambertian"))
    batch = data.collate([0])
    for _ in range(3):
        trainer.train_iteration(batch)
    model = trainer.model
    params = [p for p in model.parameters() if p.requires_grad]
    snap = [p.detach().clone() for p in params]
    nat = NativeAlbedoStep(trainer, res, res)
    assert nat.table.dtype == torch.bfloat16 and nat.d_enc.dtype == torch.bfloat16
    nat.prologue(batch["pose"], batch["intrinsics"], 11, 1234)
    nat.body()
    nat.embedding_backward()
    torch.cuda.synchronize()
    got = [p.grad.detach().clone() for p in params]
    got_count, got_loss = nat.counter.clone(), nat.loss.clone()
    assert int(got_count[0]) > 0

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
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = trainer.train_step(eager, "albedo", 1.0, text_z)[2]
        trainer.backward_only(loss)
    finally:
        model.device_count_march = False
        del model.march_noises
        del trainer.guidance.sds_grad
    torch.cuda.synchronize()
    assert torch.equal(model.last_counter, got_count)
    assert torch.equal(loss.detach().float(), got_loss)
    for p, g in zip(params, got):
        assert p.grad is not None
        assert torch.equal(p.grad, g), (tuple(p.shape), float((p.grad - g).abs().max()))


def test_native_bf16_graph_training_runs_at_c5_resolution(gpu):
    import bench
    trainer, data = bench.make_trainer(256, 9, 0, 1, True, graph=True, bf16=True)
    model = trainer.model
    before = [p.detach().clone() for p in model.parameters() if p.requires_grad]
    losses = [float(trainer.train_iteration(data.collate([i % 4]))) for i in range(20)]
    assert len(trainer._graphs) == 1
    g = next(iter(trainer._graphs.values()))
    assert g.native is not None and g.native.N == 65536
    assert all(np.isfinite(losses))
    assert int(model.step_counter[:, 0].min()) > 0
    for a, b in zip([p.detach() for p in model.parameters() if p.requires_grad], before):
        assert torch.isfinite(a).all()
        assert not torch.equal(a, b)
