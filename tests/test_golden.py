"""Golden fixtures (tests/golden/golden.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces the committed vectors bit for bit (guards the
restatement against drift).  GPU: the HIP kernels, called through the
reference-signature shims (`_raymarching`, `_gridencoder`, `_freqencoder`),
match the same vectors — bit-exact for counts / samples / indices / bits /
f32 and f16 grid features, 1e-4 rel for compositing, f32 tolerance for the
float sums.  Parity against the reference itself is unpinned.
"""
from pathlib import Path

import numpy as np
import pytest
import torch

import oracle

G = np.load(Path(__file__).resolve().parent / "golden" / "golden.npz")


def _eq(a, b):
    np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


# ------------------------------------------------------------------ CPU: oracle == golden

def test_oracle_reproduces_march():
    counts, x, d, dl = oracle.march_rays_train(G["rays_o"], G["rays_d"], G["bitfield"], 1.0, 0.0,
                                               512, 1, 128, G["nears"], G["fars"], G["noises"])
    _eq(counts, G["march_counts"])
    _eq(x, G["march_xyzs"])
    _eq(d, G["march_dirs"])
    _eq(dl, G["march_deltas"])
    nears, fars = oracle.near_far_from_aabb(G["rays_o"], G["rays_d"],
                                            np.array([-1, -1, -1, 1, 1, 1], np.float32), 0.2)
    _eq(nears, G["nears"])
    _eq(fars, G["fars"])


def test_oracle_reproduces_composite():
    rays = oracle.rays_from_counts(G["march_counts"])
    ws, dep, img = oracle.composite_rays_train_forward(G["comp_sigmas"], G["comp_rgbs"],
                                                       G["march_deltas"], rays, 1e-4)
    _eq(ws, G["comp_ws"])
    _eq(dep, G["comp_depth"])
    _eq(img, G["comp_image"])
    gs, gc = oracle.composite_rays_train_backward(G["comp_grad_ws"], G["comp_grad_image"],
                                                  G["comp_sigmas"], G["comp_rgbs"],
                                                  G["march_deltas"], rays, ws, img, 1e-4)
    _eq(gs, G["comp_grad_sigmas"])
    _eq(gc, G["comp_grad_rgbs"])


def test_oracle_reproduces_misc():
    _eq(oracle.morton3D(G["morton_coords"]), G["morton_indices"])
    _eq(oracle.packbits(G["pack_grid"], 1.0), G["pack_bits"])
    out, dy = oracle.grid_encode_forward(G["grid_inputs"], G["grid_embeddings"], G["grid_offsets"],
                                         float(G["grid_S"]), int(G["grid_H"]), 1, False, True)
    _eq(out, G["grid_out_f32"])
    _eq(dy, G["grid_dy_dx"])
    out16, _ = oracle.grid_encode_forward(G["grid_inputs"], G["grid_embeddings"].astype(np.float16),
                                          G["grid_offsets"], float(G["grid_S"]), int(G["grid_H"]))
    _eq(out16, G["grid_out_f16"])
    gemb = oracle.grid_encode_backward(G["grid_grad"], G["grid_inputs"], G["grid_offsets"], 2,
                                       float(G["grid_S"]), int(G["grid_H"]))
    _eq(gemb, G["grid_grad_embeddings"])
    fo = oracle.freq_encode_forward(G["freq_inputs"], 6)
    _eq(fo, G["freq_out"])
    _eq(oracle.freq_encode_backward(G["freq_grad"], fo, 3, 6), G["freq_grad_inputs"])


# ------------------------------------------------------------------ GPU: HIP == golden

def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.gpu
def test_gpu_march_and_composite_golden(gpu):
    import _raymarching
    n = G["rays_o"].shape[0]
    o, d = _t(G["rays_o"], gpu), _t(G["rays_d"], gpu)
    aabb = _t(np.array([-1, -1, -1, 1, 1, 1], np.float32), gpu)
    nears, fars = torch.empty(n, device=gpu), torch.empty(n, device=gpu)
    _raymarching.near_far_from_aabb(o, d, aabb, n, 0.2, nears, fars)
    _eq(nears.cpu(), G["nears"])
    _eq(fars.cpu(), G["fars"])
    m = n * 512
    xyzs, dirs = torch.zeros(m, 3, device=gpu), torch.zeros(m, 3, device=gpu)
    deltas = torch.zeros(m, 2, device=gpu)
    rays = torch.empty(n, 3, dtype=torch.int32, device=gpu)
    counter = torch.zeros(2, dtype=torch.int32, device=gpu)
    _raymarching.march_rays_train(o, d, _t(G["bitfield"], gpu), 1.0, 0.0, 512, n, 1, 128, m,
                                  nears, fars, xyzs, dirs, deltas, rays, counter,
                                  _t(G["noises"], gpu))
    total = int(G["march_counts"].sum())
    assert int(counter[0]) == total
    r = rays.cpu().numpy()
    _eq(r[:, 0], np.arange(n))
    _eq(r[:, 2], G["march_counts"])
    _eq(xyzs[:total].cpu(), G["march_xyzs"])
    _eq(dirs[:total].cpu(), G["march_dirs"])
    _eq(deltas[:total].cpu(), G["march_deltas"])
    # composite on the golden samples
    sig, rgb = _t(G["comp_sigmas"], gpu), _t(G["comp_rgbs"], gpu)
    ws, dep, img = (torch.empty(n, device=gpu), torch.empty(n, device=gpu),
                    torch.empty(n, 3, device=gpu))
    dl = deltas[:total].contiguous()
    _raymarching.composite_rays_train_forward(sig, rgb, dl, rays, total, n, 1e-4, ws, dep, img)
    for got, key in ((ws, "comp_ws"), (dep, "comp_depth"), (img, "comp_image")):
        np.testing.assert_allclose(got.cpu().numpy(), G[key], rtol=1e-4, atol=1e-6)
    gs, gc = torch.zeros(total, device=gpu), torch.zeros(total, 3, device=gpu)
    _raymarching.composite_rays_train_backward(_t(G["comp_grad_ws"], gpu),
                                               _t(G["comp_grad_image"], gpu), sig, rgb, dl, rays,
                                               ws, img, total, n, 1e-4, gs, gc)
    np.testing.assert_allclose(gs.cpu().numpy(), G["comp_grad_sigmas"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gc.cpu().numpy(), G["comp_grad_rgbs"], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_gpu_inference_golden(gpu):
    import _raymarching
    n = G["rays_o"].shape[0]
    alive = torch.arange(n, dtype=torch.int32, device=gpu)
    rays_t = _t(G["nears"], gpu).clone()
    rows = n * 4
    x, dr, dl = (torch.zeros(rows, 3, device=gpu), torch.zeros(rows, 3, device=gpu),
                 torch.zeros(rows, 2, device=gpu))
    _raymarching.march_rays(n, 4, alive, rays_t, _t(G["rays_o"], gpu), _t(G["rays_d"], gpu), 1.0,
                            0.0, 512, 1, 128, _t(G["bitfield"], gpu), _t(G["nears"], gpu),
                            _t(G["fars"], gpu), x, dr, dl, _t(G["inf_noises"], gpu))
    _eq(x.cpu(), G["inf_xyzs"])
    _eq(dr.cpu(), G["inf_dirs"])
    _eq(dl.cpu(), G["inf_deltas"])
    ws, dep, img = (torch.zeros(n, device=gpu), torch.zeros(n, device=gpu),
                    torch.zeros(n, 3, device=gpu))
    _raymarching.composite_rays(n, 4, 1e-4, alive, rays_t, _t(G["inf_sigmas"], gpu),
                                _t(G["inf_rgbs"], gpu), dl, ws, dep, img)
    _eq(alive.cpu(), G["inf_rays_alive"])
    np.testing.assert_allclose(rays_t.cpu().numpy(), G["inf_rays_t"], rtol=1e-6)
    for got, key in ((ws, "inf_ws"), (dep, "inf_depth"), (img, "inf_image")):
        np.testing.assert_allclose(got.cpu().numpy(), G[key], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_gpu_encoders_golden(gpu):
    import _freqencoder
    import _gridencoder
    import _raymarching
    c = _t(G["morton_coords"], gpu)
    idx = torch.empty(c.shape[0], dtype=torch.int32, device=gpu)
    _raymarching.morton3D(c, c.shape[0], idx)
    _eq(idx.cpu(), G["morton_indices"])
    bits = torch.empty(G["pack_bits"].shape[0], dtype=torch.uint8, device=gpu)
    _raymarching.packbits(_t(G["pack_grid"], gpu), bits.shape[0], 1.0, bits)  # N = bytes
    _eq(bits.cpu(), G["pack_bits"])

    x, offs = _t(G["grid_inputs"], gpu), _t(G["grid_offsets"], gpu)
    B, L, C, S, H = x.shape[0], 16, 2, float(G["grid_S"]), int(G["grid_H"])
    emb = _t(G["grid_embeddings"], gpu)
    out = torch.empty(B, L * C, device=gpu)
    dy = torch.empty(B, L * 3 * C, device=gpu)
    _gridencoder.grid_encode_forward_blc(x, emb, offs, out, B, 3, C, L, S, H, dy, 1, False)
    _eq(out.cpu(), G["grid_out_f32"])
    _eq(dy.cpu(), G["grid_dy_dx"])
    # reference signature ([L, B, C] output) in f16 and hash mode
    o16 = torch.empty(L, B, C, dtype=torch.float16, device=gpu)
    _gridencoder.grid_encode_forward(x, emb.half(), offs, o16, B, 3, C, L, S, H, None, 1, False)
    _eq(o16.transpose(0, 1).reshape(B, L * C).cpu(), G["grid_out_f16"])
    oh = torch.empty(L, B, C, device=gpu)
    _gridencoder.grid_encode_forward(x, emb, offs, oh, B, 3, C, L, S, H, None, 0, False)
    _eq(oh.transpose(0, 1).reshape(B, L * C).cpu(), G["grid_out_hash"])
    # sliced backward vs the exact f64 sums
    g = _t(G["grid_grad"], gpu)
    glbc = torch.empty(L, B, C, device=gpu)
    _gridencoder.grid_grad_blc_to_lbc(g, glbc, B, L, C)
    rows = int(G["grid_offsets"][-1])
    gemb = torch.empty(rows, C, device=gpu)
    parts = _gridencoder.grid_backward_default_parts(rows, C)
    partial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, C, parts), device=gpu)
    _gridencoder.grid_encode_backward_sliced(glbc, x, offs, gemb, rows, B, 3, C, L, S, H, 1, False,
                                             partial, parts)
    want = G["grid_grad_embeddings"]
    np.testing.assert_allclose(gemb.cpu().numpy(), want, rtol=1e-5,
                               atol=1e-6 * np.abs(want).max())

    fx = _t(G["freq_inputs"], gpu)
    fo = torch.empty(fx.shape[0], 39, device=gpu)
    _freqencoder.freq_encode_forward(fx, fx.shape[0], 3, 6, 39, fo)
    np.testing.assert_allclose(fo.cpu().numpy(), G["freq_out"], rtol=1e-4, atol=2e-6)
    gi = torch.empty(fx.shape[0], 3, device=gpu)
    _freqencoder.freq_encode_backward(_t(G["freq_grad"], gpu), _t(G["freq_out"], gpu), fx.shape[0],
                                      3, 6, 39, gi)
    np.testing.assert_allclose(gi.cpu().numpy(), G["freq_grad_inputs"], rtol=1e-4, atol=1e-4)
