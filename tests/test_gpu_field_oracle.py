"""End-to-end parity of the train-path chain on C2 inputs (128x128 rays) against
the CPU oracle chain: march -> fused grid field (k_field_fwd_fused) ->
compositing, and back: compositing backward -> field backward
(k_field_bwd) -> embedding backward (binned), every stage through the C-ABI.

Reference: nerf/network_grid.py:13-32,69-87 (field under fp16 autocast),
raymarching.cu:500-693 (compositing), gridencoder.cu:226-313 (embedding grads).
Oracle: oracle/field.py (f16-rounding restatement, exact float64 sums) on top
of oracle.c (grid encoding, compositing).

Tolerances come from f16 rounding, not from a second GPU implementation:
* grid features: bit-exact;
* MLP: an f32-accumulating GEMM (MFMA here, hipBLASLt in the reference) may
  round a layer's output to the neighbouring f16 value whenever the exact dot
  product lies within gamma_K * sum|terms| of an f16 rounding boundary, and that
  difference propagates.  oracle.field.forward_bounds / backward_bounds carry
  those windows through both passes; every GPU value must lie inside its
  window, and outside the windows (most samples) the GPU must equal the
  oracle bit for bit.  The fraction of samples that differ at all is printed;
* compositing of identical sigma/rgb: 1e-4 rel (north_star) against oracle.c;
  end to end (oracle sigma/rgb all the way): 1e-4 rel on every ray none of
  whose samples differ;
* MLP weight/bias gradients: the exact float64 sums of the f16 graph +/- the
  propagated windows + 2e-5 of sum|terms| for the f32 reduction over samples
  (the reference itself rounds these to f16: 2^-11 relative);
* embedding gradients from the GPU feature gradients: 1e-3 rel-norm against
  the oracle's f64 sum of the ORACLE feature gradients.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

import oracle
import oracle.field as of
from scenes import march_inputs

pytestmark = pytest.mark.gpu

ULP16 = 2.0 ** -10  # f16 spacing relative to the leading power of two
# f32 accumulation model of the MFMA chains (oracle.field._gamma): each
# v_mfma_f32_16x16x32_f16 rounds into its f32 accumulator once, K <= 64 is at
# most 2 instructions + the bias; 8 f32 roundings' worth of sum|terms| is the
# window for the forward, whose operands are normal f16 values.  (The
# order-free bound (K + 2) u also holds but opens most windows.)
MFMA_ULPS = 8


def ulp16(v):
    """Spacing of f16 values at |v| (subnormal floor 2^-24)."""
    a = np.abs(np.asarray(v, np.float64))
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -14)))
    return np.exp2(e) * ULP16


def _setup(gpu, seed, emb_scale):
    from gridencoder import GridEncoder
    torch.manual_seed(seed)
    enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                      log2_hashmap_size=16, desired_resolution=2048, gridtype="tiled").to(gpu)
    with torch.no_grad():
        enc.embeddings.uniform_(-emb_scale, emb_scale)
    layers = nn.ModuleList([nn.Linear(32, 64), nn.Linear(64, 64), nn.Linear(64, 4)]).to(gpu)
    return enc, layers


def _march(gpu, res, seed):
    import raymarching
    rays_o, rays_d, nears, fars, _, bf = march_inputs(res, res, seed=seed, noise=0.01)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
    counter = torch.zeros(2, dtype=torch.int32, device=gpu)
    xyzs, dirs, deltas, rays = raymarching.march_rays_train(
        T(rays_o), T(rays_d), 1.0, T(bf), 1, 128, T(nears), T(fars), counter, -1, False, 128,
        True, 0.0, 512)
    m = int(rays[:, 2].sum())
    return xyzs[:m].contiguous(), deltas[:m].contiguous(), rays, m


def _unperm(enc_perm):
    """The fused path stores features permuted (csrc/field_common.h
    perm_feature); back to the natural [M, 32] = (level, channel) order."""
    p = np.arange(32)
    perm = 2 * (4 * ((p & 7) >> 1) + (p >> 3)) + (p & 1)
    out = np.empty_like(enc_perm)
    out[:, perm] = enc_perm
    return out


@pytest.mark.parametrize("seed,emb_scale", [(0, 0.5), (1, 1e-4)])
def test_field_chain_matches_oracle(gpu, seed, emb_scale):
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
    table = enc_mod.embeddings.detach().half().contiguous()
    offsets = enc_mod.offsets
    ws = [p.detach().float().contiguous() for lin in layers for p in (lin.weight, lin.bias)]
    ws_np = [w.cpu().numpy() for w in ws]

    # ---- forward: fused grid field
    enc = torch.empty(M, 32, device=gpu, dtype=torch.half)
    sigma = torch.empty(M, device=gpu)
    albedo = torch.empty(M, 3, device=gpu, dtype=torch.half)
    _fieldmlp.grid_field_forward(xyzs, 1.0, table, offsets, S, Hb, gt, False, ws, enc, sigma,
                                 albedo, None)
    x_np = xyzs.cpu().numpy()
    want_enc = of.encode(x_np, 1.0, enc_mod.embeddings.detach().cpu().numpy(),
                         offsets.cpu().numpy(), S, Hb)
    got_enc = _unperm(enc.cpu().numpy())
    assert np.array_equal(got_enc.view(np.uint16), want_enc.view(np.uint16)), "features differ"

    fo = of.field_forward(x_np, ws_np, want_enc)
    fb = of.forward_bounds(fo, ws_np, acc_ulps=MFMA_ULPS)
    s_g, a_g = sigma.cpu().numpy(), albedo.cpu().numpy()
    dlog = np.abs(np.log(s_g.astype(np.float64)) - np.log(fo["sigma"].astype(np.float64)))
    assert np.all(dlog <= fb["dlog_sigma"]), \
        f"sigma outside its window: worst excess {(dlog - fb['dlog_sigma']).max():.3e}"
    da = np.abs(a_g.astype(np.float64) - fo["albedo"].astype(np.float64))
    assert np.all(da <= fb["dalbedo"]), \
        f"albedo outside its window: worst excess {(da - fb['dalbedo']).max():.3e}"
    # sigma differs beyond expf / f32 noise <=> its h0 took the other f16 value
    s_flip = dlog > 8 * 2.0 ** -24 * np.maximum(np.abs(fo["y"].astype(np.float64)), 1.0)
    a_flip = (a_g != fo["albedo"]).any(1)
    flips = s_flip | a_flip
    windowed = (fb["dh"] > 0).any(1)
    print(f"\nM={M}: h0 differs (via sigma) {s_flip.mean():.2e}, albedo differs "
          f"{a_flip.mean():.2e}, h window open {windowed.mean():.2e}")

    # ---- compositing: stage parity and end to end
    rgb = albedo.float()
    wsum = torch.empty(N, device=gpu)
    depth = torch.empty(N, device=gpu)
    image = torch.empty(N, 3, device=gpu)
    _raymarching.composite_rays_train_forward(sigma, rgb, deltas, rays, M, N, 1e-4, wsum, depth,
                                              image)
    d_np, r_np = deltas.cpu().numpy(), rays.cpu().numpy()
    ow, od, oi = oracle.composite_rays_train_forward(s_g, a_g.astype(np.float32), d_np, r_np)
    np.testing.assert_allclose(image.cpu().numpy(), oi, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(wsum.cpu().numpy(), ow, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(depth.cpu().numpy(), od, rtol=1e-4, atol=1e-5)
    ew, _, ei = oracle.composite_rays_train_forward(fo["sigma"], fo["albedo"].astype(np.float32),
                                                    d_np, r_np)
    ray_of = np.repeat(r_np[:, 0], r_np[:, 2])  # ray id of each (ray-ordered) sample
    clean = np.ones(N, bool)
    clean[np.unique(ray_of[flips])] = False
    gi, gw = image.cpu().numpy(), wsum.cpu().numpy()
    np.testing.assert_allclose(gi[clean], ei[clean], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(gw[clean], ew[clean], rtol=1e-4, atol=1e-6)
    # rays holding a flipped sample: a one-ulp change of one sample's h
    assert np.abs(gi - ei).max() <= 2e-3 and np.abs(gw - ew).max() <= 2e-3
    print(f"rays with a flipped sample: {(~clean).mean():.2e}; "
          f"max |image - oracle| {np.abs(gi - ei).max():.2e}")

    # ---- backward
    g = torch.Generator(device="cpu").manual_seed(seed + 10)
    g_img = (torch.randn(N, 3, generator=g) * 1e-2).to(gpu)
    g_ws = (torch.randn(N, generator=g) * 1e-2).to(gpu)
    gs = torch.zeros(M, device=gpu)
    grgb = torch.zeros(M, 3, device=gpu)
    _raymarching.composite_rays_train_backward(g_ws, g_img, sigma, rgb, deltas, rays, wsum, image,
                                               M, N, 1e-4, gs, grgb)
    ogs, ogc = oracle.composite_rays_train_backward(
        g_ws.cpu().numpy(), g_img.cpu().numpy(), s_g, a_g.astype(np.float32), d_np, r_np,
        wsum.cpu().numpy(), image.cpu().numpy())
    np.testing.assert_allclose(gs.cpu().numpy(), ogs, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(grgb.cpu().numpy(), ogc, rtol=1e-4, atol=1e-7)

    d_enc = torch.empty(16, M, 2, device=gpu, dtype=torch.half)
    partial = torch.empty(_fieldmlp.backward_parts(M) * _fieldmlp.params_count(), device=gpu)
    grads = [torch.empty_like(w) for w in ws]
    rows = int(offsets[-1].item())
    grad_emb = torch.empty(rows, 2, device=gpu)
    _fieldmlp.grid_field_backward(enc, xyzs, 1.0, ws, gs, grgb, d_enc, partial, grads, offsets,
                                  rows, S, Hb, gt, False, None, None, 1, None)
    gs_np, grgb16 = gs.cpu().numpy(), grgb.cpu().numpy().astype(np.float16)
    bo = of.field_backward(fo, ws_np, gs_np, grgb16)
    # backward: the order-free (K + 2) u model.  With f16-subnormal operands
    # (upstream gradients ~1e-5) the MFMA sums were measured up to ~22 u of
    # sum|terms| off the exact value (tools/field_bwd_probe.py), beyond the
    # forward's few-rounding model but inside the order-free bound.
    bb = of.backward_bounds(fo, bo, ws_np, fb, acc_ulps=None)
    d_want = bo["d_enc"]
    d_got = d_enc.cpu().numpy().transpose(1, 0, 2).reshape(M, 32)
    dd = np.abs(d_got.astype(np.float64) - d_want.astype(np.float64))
    # subnormal-range allowance: feature gradients whose exact value lies in
    # the f16 subnormal range (< 2^-14) may differ by ONE subnormal ulp
    # (2^-24) beyond the propagated windows.  Measured: ~1e-6 of elements at
    # upstream gradients ~1e-5 (tools/field_bwd_probe.py); isolated MFMA and
    # f32 -> f16 conversions of subnormals are exact / within 2 u
    # (tools/micro/f16_subnormal.hip), so the source is still open.
    sub = np.abs(d_want.astype(np.float64)) < 2.0 ** -14
    bb["d_enc"] = bb["d_enc"] + np.where(sub, 2.0 ** -24, 0.0)
    assert np.all(dd <= bb["d_enc"]), \
        f"feature grads outside their window: worst excess {(dd - bb['d_enc']).max():.3e}"
    rel = np.linalg.norm(d_got.astype(np.float64) - d_want) / np.linalg.norm(d_want)
    print(f"feature grads: differing {(dd > 0).mean():.2e}, window open "
          f"{(bb['d_enc'] > 0).mean():.2e}, rel-norm {rel:.2e}")
    assert rel <= 1e-3, rel
    for i, (a, b, w) in enumerate(zip(grads, bo["grads"], bb["grads"])):
        a = a.cpu().numpy().astype(np.float64).reshape(b.shape)
        err = np.abs(a - b)
        assert np.all(err <= w), f"param {i}: worst excess {(err - w).max():.3e}"
        print(f"param {i}: max err / max |g| {err.max() / max(np.abs(b).max(), 1e-30):.2e}")

    # ---- embedding gradient from the GPU feature gradients (binned backward)
    ne, nc, npf = _gridencoder.grid_backward_binned_scratch(M, enc_mod.offsets_host, 16, 2)
    scratch = (torch.empty(ne, device=gpu, dtype=torch.int32),
               torch.empty(nc, device=gpu, dtype=torch.int32), torch.empty(npf, device=gpu))
    launch = _gridencoder.binned_launcher(d_enc, xyzs, 1.0, offsets, enc_mod.offsets_host,
                                          grad_emb, M, None, 3, 2, 16, S, Hb, gt, False, *scratch)
    launch()
    x01 = ((x_np + np.float32(1)) / np.float32(2)).astype(np.float32)
    e_want = oracle.grid_encode_backward(d_want.reshape(M, 16, 2).astype(np.float32), x01,
                                         offsets.cpu().numpy(), 2, S, Hb)
    e_got = grad_emb.cpu().numpy().astype(np.float64)
    rel = np.linalg.norm(e_got - e_want) / max(np.linalg.norm(e_want), 1e-30)
    assert rel <= 1e-3, f"embedding grads rel-norm {rel:.3e}"


def test_ray_head_matches_oracle(gpu):
    """Background MLP + mix + depth + mask (csrc/head.hip) against
    oracle.field.bg_forward / ray_tail; background weight gradients against the
    exact f16-graph sums; grad_ws = -sum_c g_c bg_c."""
    from nerf import head as _head
    torch.manual_seed(3)
    N = 16384
    l1, l2 = nn.Linear(39, 64).to(gpu), nn.Linear(64, 3).to(gpu)
    g = torch.Generator(device="cpu").manual_seed(4)
    d = torch.randn(N, 3, generator=g)
    d = (d / d.norm(dim=1, keepdim=True)).to(gpu)
    ws = torch.rand(N, generator=g).to(gpu)
    depth = (torch.rand(N, generator=g) * 2).to(gpu)
    image = torch.rand(N, 3, generator=g).to(gpu)
    nears = (torch.rand(N, generator=g) * 0.5 + 0.2).to(gpu)
    fars = nears + (torch.rand(N, generator=g) * 2 - 0.1).to(gpu)
    ws.requires_grad_(True)
    image.requires_grad_(True)
    out_img, out_depth, mask = _head.ray_head(ws, depth, image, d, nears, fars, None, (l1, l2))
    wts = [t.detach().cpu().numpy() for t in (l1.weight, l1.bias, l2.weight, l2.bias)]
    bo = of.bg_forward(d.cpu().numpy(), wts)
    ei, ed, em = of.ray_tail(ws.detach().cpu().numpy(), depth.cpu().numpy(),
                             image.detach().cpu().numpy(), nears.cpu().numpy(),
                             fars.cpu().numpy(), bo["bg"].astype(np.float32))
    gi = out_img.detach().t().cpu().numpy()
    # colour: (1 - ws) times the background's f16 window, plus the f32 mix
    bb = of.bg_bounds(bo, wts, acc_ulps=None)  # VALU fmaf chains: order-free bound
    one_m = (1.0 - ws.detach().cpu().numpy().astype(np.float64))[:, None]
    win = one_m * bb["dbg"] + 2 * 2.0 ** -24 * np.abs(ei)
    diff = np.abs(gi.astype(np.float64) - ei)
    assert np.all(diff <= win), f"colour outside its window: {(diff - win).max():.3e}"
    print(f"\nbackground colour differs on {(diff > 0).any(1).mean():.2e} of rays")
    np.testing.assert_array_equal(out_depth.detach().cpu().numpy(), ed)
    np.testing.assert_array_equal(mask.cpu().numpy(), em)
    gimg = torch.randn(3, N, generator=g).to(gpu) * 1e-2
    grads = torch.autograd.grad(out_img, [ws, image, l1.weight, l1.bias, l2.weight, l2.bias],
                                gimg)
    gimg_np = gimg.t().cpu().numpy().astype(np.float32)
    np.testing.assert_array_equal(grads[1].cpu().numpy(), gimg_np)
    want_ws = -(gimg_np.astype(np.float64) * bo["bg"].astype(np.float64)).sum(1)
    np.testing.assert_allclose(grads[0].cpu().numpy(), want_ws, rtol=2e-3, atol=1e-7)
    gbg = gimg_np * (np.float32(1) - ws.detach().cpu().numpy())[:, None]
    bw = of.bg_bounds(bo, wts, gbg)
    for i, (a, b, w) in enumerate(zip(grads[2:], of.bg_backward(bo, wts, gbg), bw["grads"])):
        a = a.cpu().numpy().astype(np.float64).reshape(b.shape)
        err = np.abs(a - b)
        assert np.all(err <= w), f"bg param {i}: worst excess {(err - w).max():.3e}"
