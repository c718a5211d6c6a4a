"""Known-answer tests that pin the CPU oracle (oracle/oracle.c).

The reference ships no tests or fixtures and could not be built here
(SURVEY.md §4, §8c), so the oracle is pinned by analytic answers and by
independent float64 re-derivations of each formula (SURVEY.md §8c list of
KATs).  CPU only.
"""
import math

import numpy as np
import pytest
import torch

import oracle

FLT_MAX = np.finfo(np.float32).max


# ---------------------------------------------------------------- morton / packbits

def _interleave(x, y, z):
    out = 0
    for b in range(10):
        out |= ((x >> b) & 1) << (3 * b) | ((y >> b) & 1) << (3 * b + 1) | ((z >> b) & 1) << (3 * b + 2)
    return out


def test_morton_kat():
    got = oracle.morton3D(np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [127, 127, 127], [5, 3, 6]]))
    assert got.tolist() == [1, 2, 4, 2 ** 21 - 1, _interleave(5, 3, 6)]


def test_morton_roundtrip_full_grid():
    ax = np.arange(128, dtype=np.int32)
    c = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    idx = oracle.morton3D(c)
    assert np.array_equal(np.sort(idx), np.arange(128 ** 3))  # bijection onto [0, 128^3)
    assert np.array_equal(oracle.morton3D_invert(idx), c)
    sample = c[::9973]
    assert [int(v) for v in oracle.morton3D(sample)] == [_interleave(*map(int, r)) for r in sample]


def test_packbits_kat(rng):
    g = np.zeros(16, np.float32)
    g[1] = 1.0
    assert oracle.packbits(g, 0.5).tolist() == [0b10, 0]
    grid = rng.random((2, 4096), dtype=np.float32)
    want = np.packbits(grid.reshape(-1) > 0.37, bitorder="little")
    assert np.array_equal(oracle.packbits(grid, 0.37), want)
    # strict '>' (raymarching.cu:285)
    assert oracle.packbits(np.full(8, 0.5, np.float32), 0.5).tolist() == [0]


# ---------------------------------------------------------------- near / far

def test_near_far_kat():
    aabb = np.array([-1, -1, -1, 1, 1, 1], np.float32)
    o = np.array([[-2, 0, 0], [-2, 5, 0], [0, 0, 0], [0.5, 0.2, -3]], np.float32)
    d = np.array([[1, 0, 0], [1, 0, 0], [0, 0, 1], [0, 0, 1]], np.float32)
    nears, fars = oracle.near_far_from_aabb(o, d, aabb, 0.2)
    assert nears[0] == 1.0 and fars[0] == 3.0
    assert nears[1] == FLT_MAX and fars[1] == FLT_MAX  # miss
    assert nears[2] == np.float32(0.2) and fars[2] == 1.0  # inside: near clamped to min_near
    assert nears[3] == 2.0 and fars[3] == 4.0


def test_near_far_random_vs_float64(rng):
    o = (rng.random((2000, 3)) * 6 - 3).astype(np.float32)
    d = rng.normal(size=(2000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    nears, fars = oracle.near_far_from_aabb(o, d, np.array([-1, -1, -1, 1, 1, 1], np.float32), 0.05)
    with np.errstate(divide="ignore", invalid="ignore"):
        t0 = (-1 - o.astype(np.float64)) / d
        t1 = (1 - o.astype(np.float64)) / d
    lo = np.nanmax(np.minimum(t0, t1), 1)
    hi = np.nanmin(np.maximum(t0, t1), 1)
    hit = lo <= hi
    assert np.all((nears == FLT_MAX) == ~hit)
    np.testing.assert_allclose(nears[hit], np.maximum(lo[hit], 0.05), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(fars[hit], hi[hit], rtol=1e-5, atol=1e-5)


def test_sph_from_ray_kat():
    # from the centre, a ray along +x leaves Sphere(2) at (2,0,0): theta=pi/2 -> 0, phi=0
    c = oracle.sph_from_ray(np.zeros((2, 3), np.float32),
                            np.array([[1, 0, 0], [0, 0, 1]], np.float32), 2.0)
    np.testing.assert_allclose(c[0], [0.0, 0.0], atol=1e-6)
    np.testing.assert_allclose(c[1], [0.0, 0.5], atol=1e-6)  # phi = atan2(z, x) = pi/2


# ---------------------------------------------------------------- marching

def _march_args(n=64, seed=0, bitfield=None, H=128):
    r = np.random.default_rng(seed)
    center = r.normal(size=3)
    center = center / np.linalg.norm(center) * 1.3
    o = np.repeat(center[None], n, 0).astype(np.float32)
    tgt = r.normal(size=(n, 3)) * 0.3
    d = tgt - center
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    nears, fars = oracle.near_far_from_aabb(o, d, np.array([-1, -1, -1, 1, 1, 1], np.float32), 0.2)
    noises = r.random(n, dtype=np.float32)
    if bitfield is None:
        bitfield = np.full(H ** 3 // 8, 0xFF, np.uint8)
    return o, d, bitfield, nears, fars, noises


def test_march_full_occupancy_counts():
    o, d, bf, nears, fars, noises = _march_args()
    max_steps = 512
    counts, xyzs, dirs, deltas = oracle.march_rays_train(o, d, bf, 1.0, 0.0, max_steps, 1, 128,
                                                         nears, fars, noises)
    dt = np.float32(2 * np.float32(1.7320508075688772)) / np.float32(max_steps)
    off = 0
    for n in range(len(o)):
        t = np.float32(np.float64(dt) * np.float64(noises[n]) + np.float64(nears[n]))
        k = 0
        while t < fars[n] and k < max_steps:
            t = np.float32(t + dt)
            k += 1
        assert counts[n] == k, n
        # every emitted delta is (dt, dt) and the samples march along the ray
        seg = deltas[off:off + k]
        assert np.all(seg[:, 0] == dt)
        np.testing.assert_allclose(seg[:, 1], dt, rtol=0, atol=4e-7)  # t - last_t at |t|<4
        assert np.all(dirs[off:off + k] == d[n])
        off += k
    assert off == xyzs.shape[0]


def test_march_empty_and_half_space():
    o, d, _, nears, fars, noises = _march_args(n=128, seed=3)
    empty = np.zeros(128 ** 3 // 8, np.uint8)
    counts, xyzs, _, _ = oracle.march_rays_train(o, d, empty, 1.0, 0.0, 512, 1, 128, nears, fars,
                                                 noises)
    assert counts.sum() == 0 and xyzs.shape[0] == 0
    # occupy cells with x index >= 64 (x >= 0): every sample must have x >= -1/64
    ax = np.arange(128)
    cx, cy, cz = np.meshgrid(ax, ax, ax, indexing="ij")
    occ = np.zeros(128 ** 3, bool)
    occ[oracle.morton3D(np.stack([cx, cy, cz], -1).reshape(-1, 3))] = (cx >= 64).reshape(-1)
    bf = np.packbits(occ, bitorder="little")
    counts, xyzs, _, _ = oracle.march_rays_train(o, d, bf, 1.0, 0.0, 512, 1, 128, nears, fars, noises)
    assert counts.sum() > 0
    assert xyzs[:, 0].min() >= -1e-6


def test_march_samples_subset_of_dense_walk():
    """Skipping never emits a sample the dense walk would not (and rarely drops one)."""
    H = 128
    r = np.random.default_rng(7)
    occ = r.random(H ** 3) < 0.02
    bf = np.packbits(occ, bitorder="little")
    o, d, _, nears, fars, noises = _march_args(n=48, seed=5)
    counts, xyzs, _, _ = oracle.march_rays_train(o, d, bf, 1.0, 0.0, 512, 1, H, nears, fars, noises)
    off = 0
    # every emitted sample lies in an occupied cell
    cells = np.clip((0.5 * (xyzs.astype(np.float64) + 1) * H).astype(np.int64), 0, H - 1)
    idx = oracle.morton3D(cells.astype(np.int32))
    assert occ[idx].all()


def test_march_infer_matches_train_first_steps():
    o, d, bf, nears, fars, noises = _march_args(n=32, seed=11)
    counts, xyzs, _, deltas = oracle.march_rays_train(o, d, bf, 1.0, 0.0, 512, 1, 128, nears, fars,
                                                      np.zeros_like(noises))
    alive = np.arange(32, dtype=np.int32)
    x2, _, dl2 = oracle.march_rays(32, 8, alive, nears.copy(), o, d, 1.0, 0.0, 512, 1, 128, bf, fars,
                                   np.zeros(32, np.float32))
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
    for n in range(32):
        k = min(8, counts[n])
        assert np.array_equal(x2[n * 8:n * 8 + k], xyzs[offs[n]:offs[n] + k])
        assert np.all(dl2[n * 8 + k:(n + 1) * 8] == 0)


# ---------------------------------------------------------------- compositing

def _composite_f64(sig, rgb, dl, T_thresh):
    T, out = 1.0, np.zeros(3)
    ws = d = t = 0.0
    for i in range(len(sig)):
        a = 1 - math.exp(-sig[i] * dl[i, 0])
        w = a * T
        out += w * rgb[i]
        t += dl[i, 1]
        d += w * t
        ws += w
        T *= 1 - a
        if T < T_thresh:
            break
    return ws, d, out


def test_composite_single_sample_kat():
    sig = np.array([math.log(2.0) / 0.5], np.float32)
    rgb = np.array([[0.2, 0.4, 0.8]], np.float32)
    dl = np.array([[0.5, 0.25]], np.float32)
    ws, depth, image = oracle.composite_rays_train_forward(sig, rgb, dl, np.array([[0, 0, 1]]))
    np.testing.assert_allclose(ws, [0.5], rtol=1e-6)
    np.testing.assert_allclose(image[0], 0.5 * rgb[0], rtol=1e-6)
    np.testing.assert_allclose(depth, [0.125], rtol=1e-6)


def test_composite_random_vs_float64(rng):
    counts = rng.integers(0, 40, 50)
    rays = oracle.rays_from_counts(counts)
    m = int(counts.sum())
    sig = (rng.random(m) * 30).astype(np.float32)
    rgb = rng.random((m, 3), dtype=np.float32)
    dl = np.stack([np.full(m, 0.0068), rng.random(m) * 0.01 + 0.0068], -1).astype(np.float32)
    ws, depth, image = oracle.composite_rays_train_forward(sig, rgb, dl, rays, 1e-4)
    for n, (i, off, c) in enumerate(rays):
        w64, d64, img64 = _composite_f64(sig[off:off + c], rgb[off:off + c], dl[off:off + c], 1e-4)
        np.testing.assert_allclose(ws[i], w64, rtol=2e-4, atol=1e-6)
        np.testing.assert_allclose(image[i], img64, rtol=2e-4, atol=1e-6)
        np.testing.assert_allclose(depth[i], d64, rtol=2e-4, atol=1e-6)


def test_composite_backward_matches_autograd(rng):
    """The reference's closed-form gradient (raymarching.cu:657-667) equals
    autograd of the compositing sum when no ray terminates early."""
    counts = rng.integers(1, 20, 30)
    rays = oracle.rays_from_counts(counts)
    m = int(counts.sum())
    sig = (rng.random(m) * 5).astype(np.float32)
    rgb = rng.random((m, 3), dtype=np.float32)
    dl = np.stack([np.full(m, 0.02), np.full(m, 0.02)], -1).astype(np.float32)
    ws, depth, image = oracle.composite_rays_train_forward(sig, rgb, dl, rays, 0.0)
    g_ws = rng.normal(size=len(counts)).astype(np.float32)
    g_img = rng.normal(size=(len(counts), 3)).astype(np.float32)
    gs, gc = oracle.composite_rays_train_backward(g_ws, g_img, sig, rgb, dl, rays, ws, image, 0.0)

    s = torch.tensor(sig, dtype=torch.float64, requires_grad=True)
    c = torch.tensor(rgb, dtype=torch.float64, requires_grad=True)
    total = torch.zeros((), dtype=torch.float64)
    for i, off, k in rays:
        a = 1 - torch.exp(-s[off:off + k] * float(dl[0, 0]))
        T = torch.cumprod(torch.cat([torch.ones(1, dtype=torch.float64), 1 - a[:-1]]), 0)
        w = a * T
        total = total + float(g_ws[i]) * w.sum() + (torch.tensor(g_img[i], dtype=torch.float64) *
                                                   (w[:, None] * c[off:off + k]).sum(0)).sum()
    total.backward()
    np.testing.assert_allclose(gs, s.grad.numpy(), rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(gc, c.grad.numpy(), rtol=1e-4, atol=1e-6)


def test_composite_infer_vs_train(rng):
    """With n_step >= every count the inference compositor equals the train one
    (up to T = 1 - sum(w) vs the running product)."""
    counts = rng.integers(1, 8, 20)
    n = len(counts)
    sig = (rng.random((n, 8)) * 10).astype(np.float32)
    rgb = rng.random((n, 8, 3), dtype=np.float32)
    dl = np.zeros((n, 8, 2), np.float32)
    for i, c in enumerate(counts):
        dl[i, :c] = 0.01
    ws = np.zeros(n, np.float32)
    depth = np.zeros(n, np.float32)
    image = np.zeros((n, 3), np.float32)
    alive = np.arange(n, dtype=np.int32)
    rays_t = np.zeros(n, np.float32)
    oracle.composite_rays(n, 8, 1e-4, alive, rays_t, sig.reshape(-1), rgb.reshape(-1, 3),
                          dl.reshape(-1, 2), ws, depth, image)
    assert np.all(alive == -1)  # all rays ended inside the 8 slots (zero delta)
    flat_rays = oracle.rays_from_counts(counts)
    keep = np.concatenate([np.arange(c) + 8 * i for i, c in enumerate(counts)])
    ws2, _, img2 = oracle.composite_rays_train_forward(sig.reshape(-1)[keep], rgb.reshape(-1, 3)[keep],
                                                       dl.reshape(-1, 2)[keep], flat_rays, 1e-4)
    np.testing.assert_allclose(ws, ws2, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(image, img2, rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------- grid encoder

def _grid_setup():
    import sys
    sys.path.insert(0, "single-stable-dreamfusion_amd")
    from gridencoder.grid import level_offsets
    scale_per_level = np.exp2(np.log2(2048 / 16) / 15)
    offs = level_offsets(16, 2, 3, 16, scale_per_level, 16, False)
    S = float(np.float32(np.log2(scale_per_level)))
    return offs, S


def test_grid_offsets_match_survey():
    offs, S = _grid_setup()
    rows = np.diff(offs)
    assert offs[-1] == 903480
    assert rows[:3].tolist() == [4920, 13824, 32768] and np.all(rows[3:] == 65536)
    # level 15: 15 * S rounds to exactly 7 -> scale 2047, resolution 2048
    assert np.float32(15) * np.float32(S) == np.float32(7.0)


def _index64(q, res, hsize, gridtype=1):
    stride, idx, d = 1, 0, 0
    while d < 3 and stride <= hsize:
        idx += int(q[d]) * stride
        stride *= res + 1
        d += 1
    return idx % hsize


def test_grid_forward_lattice_point():
    offs, S = _grid_setup()
    rng = np.random.default_rng(1)
    emb = rng.normal(size=(int(offs[-1]), 2)).astype(np.float32)
    # x = (k - 0.5) / scale lands exactly on a lattice point of level l
    for lvl in (0, 5, 15):
        scale = np.float32(np.float32(np.exp2(np.float64(np.float32(lvl) * np.float32(S)))) * 16 - 1)
        res = int(np.ceil(scale)) + 1
        k = np.array([3, 7, 2])
        x = ((k - 0.5) / np.float64(scale)).astype(np.float32)
        pos = np.array([np.float32(np.float64(xi) * np.float64(scale) + 0.5) for xi in x])
        if not np.all(pos == k):
            continue  # rounding moved it off the lattice; other levels cover the KAT
        out, _ = oracle.grid_encode_forward(x[None], emb, offs, S, 16)
        row = offs[lvl] + _index64(k, res, offs[lvl + 1] - offs[lvl])
        np.testing.assert_array_equal(out[0, 2 * lvl:2 * lvl + 2], emb[row])


def test_grid_fine_levels_ignore_z():
    """Levels whose (res+1)^2 exceeds the 2^16 rows drop z from the tiled index."""
    offs, S = _grid_setup()
    emb = np.random.default_rng(2).normal(size=(int(offs[-1]), 2)).astype(np.float32)
    x = np.array([[0.3, 0.6, 0.2], [0.3, 0.6, 0.8]], np.float32)
    out, _ = oracle.grid_encode_forward(x, emb, offs, S, 16)
    for lvl in range(16):
        scale = np.float32(np.float32(np.exp2(np.float64(np.float32(lvl) * np.float32(S)))) * 16 - 1)
        res = int(np.ceil(scale)) + 1
        # z only enters through the corner weights, which sum to 1 when it is dropped
        same = np.allclose(out[0, 2 * lvl:2 * lvl + 2], out[1, 2 * lvl:2 * lvl + 2], rtol=1e-5,
                           atol=1e-6)
        assert same == ((res + 1) ** 2 > 65536), lvl


def test_grid_forward_random_vs_float64(rng):
    offs, S = _grid_setup()
    emb = rng.normal(size=(int(offs[-1]), 2)).astype(np.float32)
    x = rng.random((200, 3), dtype=np.float32)
    out, _ = oracle.grid_encode_forward(x, emb, offs, S, 16)
    for lvl in (0, 3, 9, 15):
        scale = np.float32(np.float32(np.exp2(np.float64(np.float32(lvl) * np.float32(S)))) * 16 - 1)
        res = int(np.ceil(scale)) + 1
        hs = int(offs[lvl + 1] - offs[lvl])
        for b in range(0, 200, 17):
            # the cell position in f32 as the kernel forms it (fma), the rest in f64
            p = (x[b].astype(np.float64) * np.float64(scale) + 0.5).astype(np.float32)
            g = np.floor(p).astype(np.int64)
            f = (p - g.astype(np.float32)).astype(np.float64)
            want = np.zeros(2)
            for kk in range(8):
                bits = [(kk >> dd) & 1 for dd in range(3)]
                w = np.prod([f[dd] if bits[dd] else 1 - f[dd] for dd in range(3)])
                want += w * emb[offs[lvl] + _index64(g + bits, res, hs)]
            np.testing.assert_allclose(out[b, 2 * lvl:2 * lvl + 2], want, rtol=1e-4, atol=1e-5)


def test_grid_out_of_bounds_is_zero():
    offs, S = _grid_setup()
    emb = np.ones((int(offs[-1]), 2), np.float32)
    out, dy = oracle.grid_encode_forward(np.array([[1.2, 0.5, 0.5], [0.5, -0.1, 0.5]], np.float32),
                                         emb, offs, S, 16, calc_dy_dx=True)
    assert np.all(out == 0) and np.all(dy == 0)


def test_grid_half_accumulation_is_rounded_per_corner():
    offs, S = _grid_setup()
    rng = np.random.default_rng(4)
    emb16 = rng.normal(size=(int(offs[-1]), 2)).astype(np.float16)
    x = rng.random((64, 3), dtype=np.float32)
    out16, _ = oracle.grid_encode_forward(x, emb16, offs, S, 16)
    out32, _ = oracle.grid_encode_forward(x, emb16.astype(np.float32), offs, S, 16)
    assert out16.dtype == np.float16
    # every f16 result equals f32 within the accumulated half rounding (8 adds)
    np.testing.assert_allclose(out16.astype(np.float32), out32, rtol=0, atol=8 * 2e-3)


def test_grid_backward_is_adjoint_of_forward(rng):
    """<grad_out, J emb> == <J^T grad_out, emb> (linearity in the table)."""
    offs, S = _grid_setup()
    emb = rng.normal(size=(int(offs[-1]), 2)).astype(np.float64)
    x = rng.random((100, 3), dtype=np.float32)
    out, _ = oracle.grid_encode_forward(x, emb, offs, S, 16)
    g = rng.normal(size=out.shape)
    gt = oracle.grid_encode_backward(g.astype(np.float64), x, offs, 2, S, 16)
    np.testing.assert_allclose((g * out).sum(), (gt * emb).sum(), rtol=1e-9)


def test_grid_dy_dx_matches_finite_difference(rng):
    offs, S = _grid_setup()
    emb = rng.normal(size=(int(offs[-1]), 2)).astype(np.float64)
    x = (rng.random((20, 3)) * 0.8 + 0.1).astype(np.float32)
    out, dy = oracle.grid_encode_forward(x, emb, offs, S, 16, calc_dy_dx=True)
    eps = 1e-4
    for dd in range(3):
        xp, xm = x.copy(), x.copy()
        xp[:, dd] += eps
        xm[:, dd] -= eps
        fd = (oracle.grid_encode_forward(xp, emb, offs, S, 16)[0] -
              oracle.grid_encode_forward(xm, emb, offs, S, 16)[0]) / (xp[:, dd] - xm[:, dd])[:, None]
        an = dy.reshape(20, 16, 3, 2)[:, :, dd, :].reshape(20, 32)
        # the interpolant is piecewise smooth: a few differences straddle a cell face
        close = np.isclose(an[:, :12], fd[:, :12], rtol=2e-2, atol=2e-2)
        assert close.mean() > 0.95, close.mean()


# ---------------------------------------------------------------- freq encoder

def test_freq_kat_zero():
    out = oracle.freq_encode_forward(np.zeros((1, 3), np.float32), 6)
    want = [0.0] * 3
    for _ in range(6):
        want += [0.0] * 3 + [1.0] * 3
    np.testing.assert_allclose(out[0], want, atol=1e-7)


def test_freq_random_vs_float64(rng):
    x = (rng.random((100, 3)) * 2 - 1).astype(np.float32)
    out = oracle.freq_encode_forward(x, 6)
    x64 = x.astype(np.float64)
    want = [x64]
    for k in range(6):
        want += [np.sin(2.0 ** k * x64), np.cos(2.0 ** k * x64)]
    np.testing.assert_allclose(out, np.concatenate(want, 1), atol=2e-6)
    g = rng.normal(size=out.shape).astype(np.float32)
    gi = oracle.freq_encode_backward(g, out, 3, 6)
    xt = torch.tensor(x64, requires_grad=True)
    parts = [xt]
    for k in range(6):
        parts += [torch.sin(2.0 ** k * xt), torch.cos(2.0 ** k * xt)]
    (torch.cat(parts, 1) * torch.tensor(g, dtype=torch.float64)).sum().backward()
    np.testing.assert_allclose(gi, xt.grad.numpy(), rtol=1e-4, atol=2e-4)


# ---------------------------------------------------------------- SH

def test_sh_explicit_low_degree(rng):
    """First 9 outputs written out as in shencoder.cu:50-60."""
    x = rng.normal(size=(20, 3))
    X, Y, Z = x.T
    out, _ = oracle.sh_encode(x, 3)
    want = np.stack([0.28209479177387814 + 0 * X, -0.48860251190291987 * Y, 0.48860251190291987 * Z,
                     -0.48860251190291987 * X, 1.0925484305920792 * X * Y, -1.0925484305920792 * Y * Z,
                     0.94617469575755997 * Z * Z - 0.31539156525251999, -1.0925484305920792 * X * Z,
                     0.54627421529603959 * (X * X - Y * Y)], 1)
    np.testing.assert_allclose(out, want, rtol=1e-12, atol=1e-12)


def test_sh_unit_vectors_vs_scipy(rng):
    from scipy.special import sph_harm_y
    v = rng.normal(size=(50, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    out, _ = oracle.sh_encode(v, 8)
    theta = np.arccos(v[:, 2])
    phi = np.arctan2(v[:, 1], v[:, 0])
    for l in range(8):
        for m in range(-l, l + 1):
            y = sph_harm_y(l, abs(m), theta, phi)  # includes the Condon-Shortley phase
            if m > 0:
                want = np.sqrt(2) * y.real
            elif m < 0:
                want = np.sqrt(2) * y.imag
            else:
                want = y.real
            np.testing.assert_allclose(out[:, l * l + l + m], want, atol=1e-10, err_msg=f"l={l} m={m}")


def test_sh_jacobian_finite_difference(rng):
    x = rng.normal(size=(10, 3))
    _, jac = oracle.sh_encode(x, 8)
    eps = 1e-6
    for d in range(3):
        xp, xm = x.copy(), x.copy()
        xp[:, d] += eps
        xm[:, d] -= eps
        fd = (oracle.sh_encode(xp, 8)[0] - oracle.sh_encode(xm, 8)[0]) / (2 * eps)
        np.testing.assert_allclose(jac[:, d], fd, rtol=1e-5, atol=1e-5)
