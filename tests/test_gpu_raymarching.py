"""GPU parity of the ray-marching kernels against the CPU oracle.

Bit-exact: near/far, morton, packbits, per-ray sample counts and every
emitted sample (xyz, dir, dt, depth-delta) of march_rays_train / march_rays.
Tolerance (north star: 1e-4 rel on composited RGB / sigma, plus a 1e-6
absolute floor for near-zero values): compositing forward and backward.
"""
import numpy as np
import pytest
import torch

import oracle
from scenes import AABB, camera_rays, march_inputs, sphere_grid

pytestmark = pytest.mark.gpu


def T(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


def assert_close(got, want, rtol=1e-4, atol=1e-6):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else got
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol)


# ------------------------------------------------------------------ utils

def test_near_far_bitexact(gpu):
    import raymarching
    r = np.random.default_rng(0)
    o = (r.random((5000, 3)) * 6 - 3).astype(np.float32)
    d = r.normal(size=(5000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[:50, 0] = 0.0  # axis-parallel rays: 1/0 = inf slabs
    d[50:60] = [0.0, 0.0, 1.0]
    for min_near in (0.2, 0.05):
        nears, fars = raymarching.near_far_from_aabb(T(o, gpu), T(d, gpu), T(AABB, gpu), min_near)
        wn, wf = oracle.near_far_from_aabb(o, d, AABB, min_near)
        np.testing.assert_array_equal(nears.cpu().numpy(), wn)
        np.testing.assert_array_equal(fars.cpu().numpy(), wf)


def test_near_far_empty(gpu):
    import raymarching
    e = torch.empty(0, 3, device=gpu)
    nears, fars = raymarching.near_far_from_aabb(e, e, T(AABB, gpu))
    assert nears.numel() == 0 and fars.numel() == 0


def test_sph_from_ray(gpu):
    import raymarching
    o = np.zeros((1000, 3), np.float32)
    d = np.random.default_rng(1).normal(size=(1000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    got = raymarching.sph_from_ray(T(o, gpu), T(d, gpu), 1.4)
    assert_close(got, oracle.sph_from_ray(o, d, 1.4), rtol=1e-5, atol=2e-6)


def test_morton_full_grid_bitexact(gpu):
    import raymarching
    ax = np.arange(128, dtype=np.int32)
    c = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    idx = raymarching.morton3D(T(c, gpu))
    np.testing.assert_array_equal(idx.cpu().numpy(), oracle.morton3D(c))
    back = raymarching.morton3D_invert(idx)
    np.testing.assert_array_equal(back.cpu().numpy(), c)
    # arbitrary 32-bit inputs: same integer semantics as the reference
    wild = np.random.default_rng(2).integers(0, 2 ** 31 - 1, (4096, 3)).astype(np.int32)
    np.testing.assert_array_equal(raymarching.morton3D(T(wild, gpu)).cpu().numpy(),
                                  oracle.morton3D(wild))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.float64])
def test_packbits_bitexact(gpu, dtype):
    import _raymarching
    grid = np.random.default_rng(3).random((1, 128 ** 3), dtype=np.float32) * 20
    g = T(grid, gpu, dtype)
    bf = torch.empty(128 ** 3 // 8, dtype=torch.uint8, device=gpu)
    _raymarching.packbits(g, bf.numel(), 9.5, bf)
    want = oracle.packbits(g.float().cpu().numpy(), 9.5)
    np.testing.assert_array_equal(bf.cpu().numpy(), want)


def test_packbits_unaligned_view(gpu):
    import raymarching
    grid = np.random.default_rng(4).random(1 + 8 * 1000, dtype=np.float32)
    g = T(grid, gpu)[1:].view(1, -1)  # 4-byte aligned, not 16
    bf = raymarching.packbits(g, 0.5)
    np.testing.assert_array_equal(bf.cpu().numpy(), oracle.packbits(grid[1:], 0.5))


# ------------------------------------------------------------------ march (train)

def _march_gpu(gpu, rays_o, rays_d, nears, fars, noises, bf, **kw):
    """Run the Python API with explicit noises (perturb via noise tensor)."""
    import _raymarching
    import raymarching
    # the API draws its own noise when perturb=True; drive the split kernels
    # directly to inject the oracle's noise
    n = rays_o.shape[0]
    o, d = T(rays_o, gpu), T(rays_d, gpu)
    ne, fa, no, b = T(nears, gpu), T(fars, gpu), T(noises, gpu), T(bf, gpu)
    max_steps = kw.get("max_steps", 512)
    cap = kw.get("cap", n * max_steps)
    zero_tail = kw.get("zero_tail", 128)
    rays = torch.empty(n, 3, dtype=torch.int32, device=gpu)
    counter = torch.zeros(2, dtype=torch.int32, device=gpu)
    bs = torch.empty(_raymarching.march_rays_train_scratch_ints(n), dtype=torch.int32, device=gpu)
    xyzs = torch.full((cap, 3), 7.0, device=gpu)  # poison: every returned row must be written
    dirs = torch.full((cap, 3), 7.0, device=gpu)
    deltas = torch.full((cap, 2), 7.0, device=gpu)
    if kw.get("staged", False):
        # count pass keeps the samples, emit pass copies them (native train step)
        stage = torch.full((_raymarching.march_rays_train_stage_floats(n, max_steps),), 5.0,
                           device=gpu)
        _raymarching.march_rays_train_count_staged(o, d, b, 1.0, 0.0, max_steps, n, 1, 128, ne,
                                                   fa, rays, counter, no, bs, stage)
        _raymarching.march_rays_train_emit_staged(d, max_steps, n, cap, xyzs, dirs, deltas, rays,
                                                  bs, zero_tail, stage)
        return xyzs, dirs, deltas, rays, counter
    _raymarching.march_rays_train_count(o, d, b, 1.0, 0.0, max_steps, n, 1, 128, ne, fa, rays,
                                        counter, no, bs)
    _raymarching.march_rays_train_emit(o, d, b, 1.0, 0.0, max_steps, n, 1, 128, cap, ne, fa, xyzs,
                                       dirs, deltas, rays, no, bs, zero_tail)
    return xyzs, dirs, deltas, rays, counter


@pytest.mark.parametrize("staged", [False, True])
def test_march_rays_train_bitexact_128x128(gpu, staged):
    rays_o, rays_d, nears, fars, noises, bf = march_inputs(128, 128, seed=0)
    xyzs, dirs, deltas, rays, counter = _march_gpu(gpu, rays_o, rays_d, nears, fars, noises, bf,
                                                   staged=staged)
    counts, wx, wd, wl = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, 512, 1, 128, nears,
                                                 fars, noises)
    rays = rays.cpu().numpy()
    total = int(counts.sum())
    assert total > 100_000  # a real workload, not an empty scene
    np.testing.assert_array_equal(rays[:, 0], np.arange(len(counts)))
    np.testing.assert_array_equal(rays[:, 2], counts)  # per-ray counts bit-exact
    np.testing.assert_array_equal(rays[:, 1], oracle.rays_from_counts(counts)[:, 1])
    assert counter.cpu().tolist() == [total, len(counts)]
    np.testing.assert_array_equal(xyzs[:total].cpu().numpy(), wx)
    np.testing.assert_array_equal(dirs[:total].cpu().numpy(), wd)
    np.testing.assert_array_equal(deltas[:total].cpu().numpy(), wl)
    # align tail (reference rule: m + 128 - m % 128 rows) is zero, rows beyond untouched
    m_al = total + 128 - total % 128
    assert torch.all(xyzs[total:m_al] == 0) and torch.all(deltas[total:m_al] == 0)
    assert torch.all(xyzs[m_al:m_al + 4] == 7.0)


@pytest.mark.parametrize("seed,radius,noise", [(1, 0.3, 0.0), (2, 0.8, 0.01), (3, 0.0, 0.05)])
def test_march_rays_train_bitexact_scenes(gpu, seed, radius, noise):
    rays_o, rays_d, nears, fars, noises, bf = march_inputs(64, 64, seed=seed, radius=radius,
                                                           noise=noise)
    xyzs, dirs, deltas, rays, counter = _march_gpu(gpu, rays_o, rays_d, nears, fars, noises, bf)
    counts, wx, wd, wl = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, 512, 1, 128, nears,
                                                 fars, noises)
    total = int(counts.sum())
    np.testing.assert_array_equal(rays.cpu().numpy()[:, 2], counts)
    np.testing.assert_array_equal(xyzs[:total].cpu().numpy(), wx)
    np.testing.assert_array_equal(deltas[:total].cpu().numpy(), wl)


def test_march_rays_train_edge_cases(gpu):
    """Full and empty occupancy, max_steps cap, rays that miss the box."""
    rays_o, rays_d, nears, fars, noises, _ = march_inputs(32, 32, seed=4)
    rays_o[:100] = [5.0, 5.0, 5.0]  # these miss: near = far = FLT_MAX
    nears, fars = oracle.near_far_from_aabb(rays_o, rays_d, AABB, 0.2)
    for bf, max_steps in ((np.full(128 ** 3 // 8, 255, np.uint8), 64),
                          (np.full(128 ** 3 // 8, 255, np.uint8), 1024),
                          (np.zeros(128 ** 3 // 8, np.uint8), 512)):
        xyzs, _, deltas, rays, counter = _march_gpu(gpu, rays_o, rays_d, nears, fars, noises, bf,
                                                    max_steps=max_steps)
        counts, wx, _, wl = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, max_steps, 1,
                                                    128, nears, fars, noises)
        np.testing.assert_array_equal(rays.cpu().numpy()[:, 2], counts)
        assert counts.max() <= max_steps and np.all(counts[:100] == 0)
        total = int(counts.sum())
        np.testing.assert_array_equal(xyzs[:total].cpu().numpy(), wx)
        np.testing.assert_array_equal(deltas[:total].cpu().numpy(), wl)


@pytest.mark.parametrize("staged", [False, True])
def test_march_rays_train_capacity_overflow(gpu, staged):
    """mean_count mode: rays whose samples do not fit in M are not written and
    their rows read as zero (raymarching.cu:416 + the caller's zero fill)."""
    rays_o, rays_d, nears, fars, noises, bf = march_inputs(32, 32, seed=5, radius=0.7)
    counts, wx, _, _ = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, 512, 1, 128, nears,
                                               fars, noises)
    cap = int(counts.sum()) // 2
    xyzs, _, deltas, rays, _ = _march_gpu(gpu, rays_o, rays_d, nears, fars, noises, bf, cap=cap,
                                          zero_tail=-1, staged=staged)
    offs = oracle.rays_from_counts(counts)[:, 1]
    fit = offs + counts <= cap
    written = int((offs + counts)[fit].max())
    np.testing.assert_array_equal(xyzs[:written].cpu().numpy(), wx[:written])
    assert torch.all(xyzs[written:] == 0) and torch.all(deltas[written:] == 0)


def test_march_rays_train_reference_abi(gpu):
    """The reference-signature entry point (caller-zeroed N*max_steps buffers)."""
    import _raymarching
    rays_o, rays_d, nears, fars, noises, bf = march_inputs(48, 48, seed=6)
    n = rays_o.shape[0]
    M = n * 512
    xyzs = torch.zeros(M, 3, device=gpu)
    dirs = torch.zeros(M, 3, device=gpu)
    deltas = torch.zeros(M, 2, device=gpu)
    rays = torch.empty(n, 3, dtype=torch.int32, device=gpu)
    counter = torch.zeros(2, dtype=torch.int32, device=gpu)
    _raymarching.march_rays_train(T(rays_o, gpu), T(rays_d, gpu), T(bf, gpu), 1.0, 0.0, 512, n, 1,
                                  128, M, T(nears, gpu), T(fars, gpu), xyzs, dirs, deltas, rays,
                                  counter, T(noises, gpu))
    counts, wx, _, wl = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, 512, 1, 128, nears,
                                                fars, noises)
    total = int(counts.sum())
    assert counter.cpu().tolist() == [total, n]
    # compare per ray id (the reference's row order is arrival order)
    r = rays.cpu().numpy()
    gx = xyzs.cpu().numpy()
    offs = oracle.rays_from_counts(counts)[:, 1]
    for i in range(0, n, 97):
        rid, off, c = r[i]
        assert c == counts[rid]
        np.testing.assert_array_equal(gx[off:off + c], wx[offs[rid]:offs[rid] + c])


def test_march_rays_train_api(gpu):
    """Python API: force_all_rays slicing + align rule, ordered rays, counter."""
    import raymarching
    rays_o, rays_d, nears, fars, noises, bf = march_inputs(64, 64, seed=7)
    counter = torch.zeros(2, dtype=torch.int32, device=gpu)
    xyzs, dirs, deltas, rays = raymarching.march_rays_train(
        T(rays_o, gpu), T(rays_d, gpu), 1.0, T(bf, gpu), 1, 128, T(nears, gpu), T(fars, gpu),
        counter, -1, False, 128, True, 0.0, 512)
    counts, wx, _, _ = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, 512, 1, 128, nears,
                                               fars, np.zeros_like(noises))
    m = int(counts.sum())
    assert xyzs.shape[0] == m + 128 - m % 128
    np.testing.assert_array_equal(xyzs[:m].cpu().numpy(), wx)
    assert torch.all(xyzs[m:] == 0)
    np.testing.assert_array_equal(rays[:, 2].cpu().numpy(), counts)


# ------------------------------------------------------------------ compositing

def _composite_case(gpu, seed=0, T_thresh=1e-4):
    rays_o, rays_d, nears, fars, noises, bf = march_inputs(64, 64, seed=seed, radius=0.6)
    counts, wx, _, wl = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, 512, 1, 128, nears,
                                                fars, noises)
    rays = oracle.rays_from_counts(counts)
    r = np.random.default_rng(seed)
    m = wx.shape[0]
    sig = (r.random(m) * 40).astype(np.float32)
    rgb = r.random((m, 3), dtype=np.float32)
    return rays, sig, rgb, wl


@pytest.mark.parametrize("T_thresh", [1e-4, 1e-2, 0.0])
def test_composite_train_forward_backward(gpu, T_thresh):
    import _raymarching
    import raymarching
    rays, sig, rgb, dl = _composite_case(gpu)
    n, m = rays.shape[0], sig.shape[0]
    ws, depth, img = oracle.composite_rays_train_forward(sig, rgb, dl, rays, T_thresh)
    s = T(sig, gpu).requires_grad_(True)
    c = T(rgb, gpu).requires_grad_(True)
    rt = T(rays, gpu)
    setattr(rt, "_dfhip_ray_ordered", True)
    gws, gdepth, gimg = raymarching.composite_rays_train(s, c, T(dl, gpu), rt, T_thresh)
    assert_close(gws, ws)
    assert_close(gimg, img)
    assert_close(gdepth, depth, atol=1e-5)
    r = np.random.default_rng(9)
    g_ws = r.normal(size=n).astype(np.float32)
    g_img = r.normal(size=(n, 3)).astype(np.float32)
    (gws * T(g_ws, gpu)).sum().add_((gimg * T(g_img, gpu)).sum()).backward()
    want_s, want_c = oracle.composite_rays_train_backward(g_ws, g_img, sig, rgb, dl, rays, ws, img,
                                                          T_thresh)
    assert_close(s.grad, want_s, atol=1e-5)
    assert_close(c.grad, want_c, atol=1e-6)
    # the dense (no-memset) backward equals the reference-form one
    gs0 = torch.zeros(m, device=gpu)
    gc0 = torch.zeros(m, 3, device=gpu)
    _raymarching.composite_rays_train_backward(T(g_ws, gpu), T(g_img, gpu), s.detach(), c.detach(),
                                               T(dl, gpu), rt, gws.detach(), gimg.detach(), m, n,
                                               T_thresh, gs0, gc0)
    assert torch.equal(gs0, s.grad) and torch.equal(gc0, c.grad)


def test_composite_empty_rays(gpu):
    import raymarching
    rays = torch.tensor([[0, 0, 0], [1, 0, 0]], dtype=torch.int32, device=gpu)
    s = torch.zeros(0, device=gpu)
    ws, depth, img = raymarching.composite_rays_train(s, torch.zeros(0, 3, device=gpu),
                                                      torch.zeros(0, 2, device=gpu), rays)
    assert torch.all(ws == 0) and torch.all(img == 0) and torch.all(depth == 0)


# ------------------------------------------------------------------ inference

def test_march_and_composite_infer(gpu):
    """Full inference loop on GPU vs the same loop on the oracle."""
    import raymarching
    rays_o, rays_d, nears, fars, _, bf = march_inputs(64, 64, seed=8, radius=0.6, noise=0.01)
    n = rays_o.shape[0]
    r = np.random.default_rng(8)
    # a fixed analytic field: sigma and rgb from the position
    def field(x):
        sig = 30.0 * np.exp(-4 * (x ** 2).sum(-1))
        return sig.astype(np.float32), (0.5 + 0.5 * np.sin(3 * x)).astype(np.float32)

    # oracle loop
    o_alive = np.arange(n, dtype=np.int32)
    o_t = nears.copy()
    o_ws, o_d, o_img = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
    g_alive = torch.arange(n, dtype=torch.int32, device=gpu)
    g_t = T(nears, gpu).clone()
    g_ws, g_d = torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    g_img = torch.zeros(n, 3, device=gpu)
    step = 0
    while step < 512 and len(o_alive) > 0:
        k = len(o_alive)
        n_step = max(min(n // k, 8), 1)
        ox, _, odl = oracle.march_rays(k, n_step, o_alive, o_t, rays_o, rays_d, 1.0, 0.0, 512, 1,
                                       128, bf, fars, np.zeros(k, np.float32))
        gx, _, gdl = raymarching.march_rays(k, n_step, g_alive, g_t, T(rays_o, gpu), T(rays_d, gpu),
                                            1.0, T(bf, gpu), 1, 128, T(nears, gpu), T(fars, gpu),
                                            128, False, 0.0, 512)
        rows = k * n_step
        np.testing.assert_array_equal(gx[:rows].cpu().numpy(), ox)
        np.testing.assert_array_equal(gdl[:rows].cpu().numpy(), odl)
        assert torch.all(gx[rows:] == 0)
        sig, rgb = field(ox)
        oracle.composite_rays(k, n_step, 1e-2, o_alive, o_t, sig, rgb, odl, o_ws, o_d, o_img)
        raymarching.composite_rays(k, n_step, g_alive, g_t, T(sig, gpu), T(rgb, gpu), gdl[:rows],
                                   g_ws, g_d, g_img, 1e-2)
        np.testing.assert_array_equal(g_alive.cpu().numpy(), o_alive)
        o_alive = o_alive[o_alive >= 0].copy()
        g_alive = g_alive[g_alive >= 0]
        step += n_step
    assert_close(g_ws, o_ws, atol=1e-5)
    assert_close(g_img, o_img, atol=1e-5)
