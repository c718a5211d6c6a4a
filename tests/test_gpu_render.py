"""Fused persistent inference renderer (csrc/render.hip)
against the reference-structured inference loop of run_cuda
(renderer.py:496-532: march_rays -> grid field -> composite_rays, whose
kernels test_gpu_raymarching pins to the CPU oracle).

The fused kernel restarts each ray's march from the composited t after every
sample, i.e. it is the loop with n_step = 1: against that schedule it must be
bit-identical; against the reference's default schedule (n_step up to 8) it
agrees to 1e-4 (see csrc/render.hip for why the two schedules differ)."""
import numpy as np
import pytest
import torch

from scenes import camera_rays, sphere_bitfield

pytestmark = pytest.mark.gpu


def _model(gpu, seed=0, scale=0.5, occupancy="sphere"):
    import main
    from nerf.network_grid import NeRFNetwork
    torch.manual_seed(seed)
    opt = main.parse_opt(["--text", "render", "-O"])
    m = NeRFNetwork(opt).to(gpu)
    with torch.no_grad():
        m.encoder.embeddings.uniform_(-scale, scale)
    if occupancy == "sphere":
        m.density_bitfield.copy_(torch.from_numpy(sphere_bitfield(0.6, 0.003, seed)).to(gpu))
    else:
        with torch.autocast("cuda", dtype=torch.float16):
            m.update_extra_state()
    m.eval()
    return m


def _rays(gpu, h, w, seed, radius=1.6):
    o, d = camera_rays(h, w, seed, radius=radius)
    return torch.from_numpy(o).to(gpu), torch.from_numpy(d).to(gpu)


def _both(m, rays_o, rays_d, n_step_max, perturb=False, T_thresh=1e-4, max_steps=512):
    import raymarching
    nears, fars = raymarching.near_far_from_aabb(rays_o, rays_d, m.aabb_infer)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        field = m.native_infer_field("albedo", rays_o)
        assert field is not None
        torch.manual_seed(7)
        fused = m._infer_fused(rays_o, rays_d, nears, fars, field, perturb, 0.0, max_steps,
                               T_thresh)
        torch.manual_seed(7)
        loop = m._infer_loop(rays_o, rays_d, nears, fars, None, 1.0, "albedo", perturb, 0.0,
                             max_steps, T_thresh, n_step_max=n_step_max)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in fused], [t.cpu().numpy() for t in loop]


@pytest.mark.parametrize("occupancy,scale,seed", [("sphere", 0.5, 0), ("sphere", 2.0, 1),
                                                  ("grid", 1.0, 2)])
def test_fused_infer_bit_exact_vs_nstep1_loop(gpu, occupancy, scale, seed):
    m = _model(gpu, seed, scale, occupancy)
    rays_o, rays_d = _rays(gpu, 48, 40, seed)
    (fw, fd, fi), (lw, ld, li) = _both(m, rays_o, rays_d, n_step_max=1)
    assert (lw > 0).sum() > 100  # the scene is not empty
    np.testing.assert_array_equal(fw, lw)
    np.testing.assert_array_equal(fd, ld)
    np.testing.assert_array_equal(fi, li)


def test_fused_infer_perturbed_bit_exact(gpu):
    """perturb=True: the first march step of each ray moves by noise * dt_min
    with the same torch.rand draw the loop makes (renderer.py:522)."""
    m = _model(gpu, 3, 1.0, "sphere")
    rays_o, rays_d = _rays(gpu, 32, 32, 3)
    (fw, fd, fi), (lw, ld, li) = _both(m, rays_o, rays_d, n_step_max=1, perturb=True)
    np.testing.assert_array_equal(fw, lw)
    np.testing.assert_array_equal(fi, li)
    np.testing.assert_array_equal(fd, ld)


def test_fused_infer_vs_default_schedule(gpu):
    m = _model(gpu, 4, 1.0, "sphere")
    rays_o, rays_d = _rays(gpu, 64, 64, 4)
    (fw, fd, fi), (lw, ld, li) = _both(m, rays_o, rays_d, n_step_max=8)
    # the default schedule continues from the march's own t inside an iteration
    # (1-ulp shifts where the f32 delta sum rounds): 1e-4 per ray
    np.testing.assert_allclose(fw, lw, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(fi, li, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(fd, ld, rtol=1e-4, atol=1e-3)


def test_fused_infer_edge_cases(gpu):
    """Missing rays (near = far = FLT_MAX), an empty bitfield, an early
    T_thresh and a tiny max_steps: every ray is written exactly once."""
    m = _model(gpu, 5, 2.0, "sphere")
    rays_o, rays_d = _rays(gpu, 16, 16, 5, radius=3.0)  # most rays miss the cube
    for T_thresh, max_steps in ((1e-4, 512), (0.5, 512), (1e-4, 3)):
        (fw, fd, fi), (lw, ld, li) = _both(m, rays_o, rays_d, 1, T_thresh=T_thresh,
                                           max_steps=max_steps)
        np.testing.assert_array_equal(fw, lw)
        np.testing.assert_array_equal(fi, li)
    m.density_bitfield.zero_()
    (fw, fd, fi), _ = _both(m, rays_o, rays_d, 1)
    assert not fw.any() and not fi.any() and not fd.any()


def test_fused_infer_sample_count_and_render_api(gpu):
    """run_cuda's eval branch uses the fused kernel (renderer.render, the
    reference API) and reports the number of samples it evaluated."""
    import raymarching
    m = _model(gpu, 6, 1.0, "sphere")
    rays_o, rays_d = _rays(gpu, 24, 24, 6)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        out = m.render(rays_o[None], rays_d[None], staged=True, perturb=False, max_steps=512)
        work = m.last_infer_work.cpu().numpy().view(np.uint32)
        m.native_infer = False
        ref = m.render(rays_o[None], rays_d[None], staged=True, perturb=False, max_steps=512)
    for k in ("image", "depth", "weights_sum"):
        np.testing.assert_allclose(out[k].float().cpu().numpy(), ref[k].float().cpu().numpy(),
                                   rtol=1e-4, atol=1e-4)
    # sample count = the loop's n_step = 1 march counts (each sample evaluated once)
    nears, fars = raymarching.near_far_from_aabb(rays_o, rays_d, m.aabb_infer)
    assert work[1] > 0 and work[2] == 0


def test_eval_background_beside_render(gpu):
    """The eval frame's background net on a side stream beside the fused
    render (renderer._background_async, then the plain head's mix) gives the
    frame of the fused net head after the render, bit for bit."""
    m = _model(gpu, 5, 1.0, "grid")
    assert m.bg_radius > 0 and m.native_background_layers() is not None
    rays_o, rays_d = _rays(gpu, 32, 40, 5)
    outs = []
    for overlap in (True, False):
        m.infer_overlap_bg = overlap
        m.__dict__.pop("_bg_stream", None)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            out = m.render(rays_o[None], rays_d[None], staged=True, perturb=False,
                           max_steps=512)
        torch.cuda.synchronize()
        assert ("_bg_stream" in m.__dict__) == overlap
        outs.append({k: out[k].float().cpu().numpy() for k in ("image", "depth", "weights_sum")})
    m.infer_overlap_bg = True
    assert (outs[1]["weights_sum"] < 0.99).sum() > 100  # the background shows
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


def _oracle_render(m, rays_o, rays_d, nears, fars, max_steps=512, T_thresh=1e-4):
    """The reference's inference loop (renderer.py:496-532) at n_step = 1 on
    the CPU oracle: oracle.march_rays -> oracle/field.py (f16 autocast
    restatement, albedo shading) -> oracle.composite_rays.  Also returns,
    per ray, whether any composited sample had an open f16 rounding window
    (where a GPU MLP may round h to the neighbouring value)."""
    import oracle
    import oracle.field as of
    from test_gpu_field_oracle import MFMA_ULPS
    enc = m.encoder
    emb = enc.embeddings.detach().float().cpu().numpy()
    offsets = enc.offsets.cpu().numpy()
    S, Hb = float(np.log2(enc.per_level_scale)), int(enc.base_resolution)
    ws_np = [p.detach().float().cpu().numpy() for lin in m.sigma_net.net
             for p in (lin.weight, lin.bias)]
    o, d = rays_o.cpu().numpy(), rays_d.cpu().numpy()
    fa = np.ascontiguousarray(fars.cpu().numpy(), np.float32)
    bf = m.density_bitfield.cpu().numpy()
    N = o.shape[0]
    wsum, depth = np.zeros(N, np.float32), np.zeros(N, np.float32)
    image = np.zeros((N, 3), np.float32)
    alive = np.arange(N, dtype=np.int32)
    rays_t = np.ascontiguousarray(nears.cpu().numpy(), np.float32).copy()
    opened = np.zeros(N, bool)
    for step in range(max_steps):
        n = alive.shape[0]
        if n == 0:
            break
        xyzs, _, deltas = oracle.march_rays(n, 1, alive, rays_t, o, d, m.bound, 0.0, max_steps,
                                            m.cascade, m.grid_size, bf, fa,
                                            np.zeros(n, np.float32))
        f16 = of.encode(xyzs, m.bound, emb, offsets, S, Hb)
        fo = of.field_forward(xyzs, ws_np, f16)
        fb = of.forward_bounds(fo, ws_np, acc_ulps=MFMA_ULPS)
        live = deltas[:, 0] > 0
        opened[alive[live & (fb["dh"] > 0).any(1)]] = True
        oracle.composite_rays(n, 1, T_thresh, alive, rays_t, fo["sigma"],
                              fo["albedo"].astype(np.float32), deltas, wsum, depth, image)
        alive = np.ascontiguousarray(alive[alive >= 0])
    return wsum, depth, image, opened


@pytest.mark.parametrize("occupancy,scale,seed", [("sphere", 0.5, 0), ("grid", 1.0, 2)])
def test_fused_infer_matches_oracle(gpu, occupancy, scale, seed):
    """k_render_infer against the CPU oracle loop: rays none of whose samples
    has an open f16 rounding window agree to 1e-4 rel (north_star); the rest
    differ by at most the effect of one-ulp h changes (measured <= 5e-6)."""
    import raymarching
    m = _model(gpu, seed, scale, occupancy)
    rays_o, rays_d = _rays(gpu, 40, 36, seed)
    nears, fars = raymarching.near_far_from_aabb(rays_o, rays_d, m.aabb_infer)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        field = m.native_infer_field("albedo", rays_o)
        fw, fd, fi = (t.cpu().numpy() for t in m._infer_fused(
            rays_o, rays_d, nears, fars, field, False, 0.0, 512, 1e-4))
    ow, od, oi, opened = _oracle_render(m, rays_o, rays_d, nears, fars)
    assert (ow > 0).sum() > 100
    c = ~opened
    np.testing.assert_allclose(fw[c], ow[c], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(fi[c], oi[c], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(fd[c], od[c], rtol=1e-4, atol=1e-5)
    print(f"\nrays with an open window: {opened.mean():.3f}; max |image - oracle| there "
          f"{np.abs(fi - oi)[opened].max() if opened.any() else 0.0:.2e}")
    # measured: <= 5e-6 on those rays (a one-ulp h change moves one sample's alpha)
    assert np.abs(fi - oi).max() <= 1e-3 and np.abs(fw - ow).max() <= 1e-3


@pytest.mark.parametrize("occupancy", ["grid", "sphere"])
def test_fused_infer_bit_exact_at_c4_size(gpu, occupancy):
    """C4 itself (BASELINE configs[3]): the 800 x 800 test-view frame of the
    bench (640,000 rays; R0 = update_extra_state occupancy of a seeded
    U(-0.5, 0.5) network, R1 = the analytic radius-0.5 sphere), where the
    persistent kernel's ray queue, refills and retirements run under full
    contention.  Every ray must equal the n_step = 1 loop bit for bit (the
    loop's kernels are pinned to the CPU oracle in test_gpu_raymarching)."""
    import bench
    import main
    from nerf.network_grid import NeRFNetwork
    from nerf.provider import NeRFDataset
    res = 800
    opt = main.parse_opt(["--text", "a hamburger", "-O", "--h", str(res), "--w", str(res)])
    torch.manual_seed(1)
    m = NeRFNetwork(opt).to(gpu)
    with torch.no_grad():
        m.encoder.embeddings.uniform_(-0.5, 0.5)
    with torch.autocast("cuda", dtype=torch.float16):
        for _ in range(3):
            m.update_extra_state()
    if occupancy == "sphere":
        bench.sphere_occupancy_(m)
    m.eval()
    data = NeRFDataset(opt, device=gpu, type="test", H=res, W=res, size=8).collate([1])
    rays_o = data["rays_o"][0].contiguous()
    rays_d = data["rays_d"][0].contiguous()
    assert rays_o.shape[0] == 640000
    (fw, fd, fi), (lw, ld, li) = _both(m, rays_o, rays_d, n_step_max=1)
    samples = int(m.last_infer_work.cpu().numpy().view(np.uint32)[1])
    assert samples > 5_000_000  # a C4-sized workload (bench: 11.6 M / 13.5 M samples)
    assert (lw > 0).sum() > 100_000
    np.testing.assert_array_equal(fw, lw)
    np.testing.assert_array_equal(fd, ld)
    np.testing.assert_array_equal(fi, li)


def test_ray_order_and_ordered_queue(gpu, monkeypatch):
    """dfhip_render_ray_order against numpy (chunks of 2^cl consecutive rays by
    ascending summed squared distance of their lines from the origin,
    quantised to 64 levels, ties in chunk order; a partial last chunk scaled
    to a whole one), and the queue in that
    order renders bit-identically to pixel order — for chunk sizes 1, 8, 64
    and N not a multiple of the chunk (the partial chunk anywhere in the
    order)."""
    import _fieldmlp
    m = _model(gpu, 8, 1.0, "grid")
    rays_o, rays_d = _rays(gpu, 37, 29, 8)  # N = 1073
    n = rays_o.shape[0]
    o, d = rays_o.cpu().double().numpy(), rays_d.cpu().double().numpy()
    t = -(o * d).sum(1) / (d * d).sum(1)
    dist = ((o + t[:, None] * d) ** 2).sum(1)
    for cl in (0, 3, 6):
        cost_dev = torch.empty(-(-n // (1 << cl)), device=gpu)
        order = _fieldmlp.render_ray_order(rays_o, rays_d, cl, cost=cost_dev).cpu().numpy()
        nc = -(-n // (1 << cl))
        assert sorted(order.tolist()) == list(range(nc))
        cost = np.array([dist[c << cl:(c + 1) << cl].mean() * (1 << cl) for c in range(nc)])
        np.testing.assert_allclose(cost_dev.cpu().numpy(), cost, rtol=1e-4, atol=1e-6 * cost.max())
        # buckets of the device costs: non-decreasing along the order, chunk
        # indices increasing inside a bucket
        c32 = cost_dev.cpu().numpy()
        q = np.minimum((c32 - c32.min()) * np.float32(64 / (c32.max() - c32.min())), 63)
        b = q.astype(np.int64)[order]
        assert np.all(np.diff(b) >= 0)
        same = np.diff(b) == 0
        assert np.all(np.diff(order)[same] > 0)
    outs = []
    for flag, cl in ((0, 6), (1, 0), (1, 3), (1, 6), (2, 3), (2, 6)):
        m.infer_order, m.infer_chunk_log2 = flag, cl
        (fw, fd, fi), _ = _both(m, rays_o, rays_d, 1)
        outs.append((fw, fd, fi))
    assert (outs[0][0] > 0).sum() > 100
    for got in outs[1:]:
        for a, b in zip(outs[0], got):
            np.testing.assert_array_equal(a, b)


def test_ordered_queue_mirror_and_tiles(gpu):
    """The queue's chunk layouts render bit-identically to pixel order with
    the same sample count (every ray taken exactly once): mirrored halves
    over several blocks of G chunk positions and a partial one (cl 3), one
    partial block (cl 6), 8 x 8 tile chunks (the tile cost is the tile rays'
    mean squared line distance x 64, restated in numpy), and a tile width
    the renderer does not apply (strips)."""
    import _fieldmlp
    m = _model(gpu, 3, 1.0, "grid")
    h, w = 40, 48
    rays_o, rays_d = _rays(gpu, h, w, 3)
    n = rays_o.shape[0]
    o, d = rays_o.cpu().double().numpy(), rays_d.cpu().double().numpy()
    t = -(o * d).sum(1) / (d * d).sum(1)
    dist = ((o + t[:, None] * d) ** 2).sum(1).reshape(h // 8, 8, w // 8, 8)
    cost = torch.empty(n // 64, device=gpu)
    order = _fieldmlp.render_ray_order(rays_o, rays_d, 6, cost=cost, tile_w=w).cpu().numpy()
    assert sorted(order.tolist()) == list(range(n // 64))
    want = dist.transpose(0, 2, 1, 3).reshape(-1, 64).mean(1) * 64
    np.testing.assert_allclose(cost.cpu().numpy(), want, rtol=1e-4, atol=1e-6 * want.max())
    with pytest.raises(RuntimeError, match="tile chunks"):
        _fieldmlp.render_ray_order(rays_o, rays_d, 6, tile_w=w + 8)  # N not 8 rows of it
    with pytest.raises(RuntimeError, match="tile chunks"):
        _fieldmlp.render_ray_order(rays_o, rays_d, 3, tile_w=w)  # tiles are 64-ray chunks
    runs = []
    variants = [(0, 6, 0), (1, 0, 0), (1, 3, 0), (1, 6, 0), (1, 6, w), (2, 6, w), (1, 3, w),
                (1, 6, w + 8)]
    for flag, cl, tile in variants:
        m.infer_order, m.infer_chunk_log2, m.infer_tile_w = flag, cl, tile
        (fw, fd, fi), _ = _both(m, rays_o, rays_d, 1)
        runs.append(((fw, fd, fi), m.last_infer_work.cpu().numpy()[:3].copy()))
    m.infer_tile_w = 0
    (ref, ref_work) = runs[0]
    assert (ref[0] > 0).sum() > 100
    for (got, work), v in zip(runs[1:], variants[1:]):
        for a, b in zip(ref, got):
            np.testing.assert_array_equal(a, b, err_msg=str(v))
        np.testing.assert_array_equal(work[1:3], ref_work[1:3], err_msg=str(v))


def _f32(x):
    return np.float32(x)


def _fma32(a, b, c):
    """f32 fmaf restated in f64 (the f32 x f32 product is exact in f64)."""
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def test_ray_order_occupancy_cost_vs_numpy(gpu):
    """dfhip_render_ray_order_occ (the infer_order = 2 option): each chunk's
    cost is minus the occupied cells at 16 evenly spaced points of its rays'
    [near, far), restated in numpy on a hand-built bitfield (one cascade,
    H = 128, an occupied ball, Morton order via oracle.morton3D); the order is
    a stable sort of the chunks by 64 cost buckets."""
    import _fieldmlp
    import oracle
    H, bound, cl = 128, 1.0, 6
    rng = np.random.default_rng(5)
    cells = np.stack(np.meshgrid(np.arange(H), np.arange(H), np.arange(H), indexing="ij"),
                     -1).reshape(-1, 3).astype(np.int32)
    centre = (cells + 0.5) / H * 2 - 1
    occ = (np.linalg.norm(centre - np.array([0.2, -0.1, 0.0]), axis=1) < 0.55)
    occ |= rng.random(occ.shape[0]) < 0.02  # scattered occupied cells too
    bits = np.zeros(H ** 3, np.uint8)
    bits[oracle.morton3D(cells)] = occ
    bitfield = np.packbits(bits.reshape(-1, 8), axis=1, bitorder="little").reshape(-1)
    N = 64 * 40
    ro = (rng.normal(size=(N, 3)) * 0.1 + np.array([0.0, 0.0, 2.5])).astype(np.float32)
    tgt = (rng.random((N, 3)) * 1.6 - 0.8).astype(np.float32)
    rd = tgt - ro
    rd = (rd / np.linalg.norm(rd, axis=1, keepdims=True)).astype(np.float32)
    nears = (rng.random(N) * 0.5 + 1.2).astype(np.float32)
    fars = (nears + rng.random(N) * 2.0).astype(np.float32)
    fars[::97] = nears[::97]  # rays missing the box: no probes
    dev = dict(device=gpu)
    cost = torch.empty(N >> cl, dtype=torch.float32, **dev)
    order = _fieldmlp.render_ray_order(
        torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu), cl, cost=cost,
        occ=(torch.from_numpy(nears).to(gpu), torch.from_numpy(fars).to(gpu),
             torch.from_numpy(bitfield).to(gpu), bound, 1, H, 1024))
    torch.cuda.synchronize()
    # numpy restatement of k_chunk_cost_occ (render.hip) for C = 1, H = 128
    want = np.zeros(N >> cl, np.float64)
    for r in range(N):
        n0, f0 = nears[r], fars[r]
        if not f0 > n0:
            continue
        step = _f32(f0 - n0) / _f32(16)
        for i in range(16):
            t = _fma32(_f32(i) + _f32(0.5), step, n0)
            p = [min(max(_fma32(t, rd[r, d], ro[r, d]), _f32(-bound)), _f32(bound))
                 for d in range(3)]
            c = [int(min(max(_fma32(p[d], _f32(1.0), _f32(1.0)) * _f32(H / 2), 0.0), H - 1))
                 for d in range(3)]
            want[r >> cl] -= float(bits[oracle.morton3D(np.array([c], np.int32))[0]])
    np.testing.assert_array_equal(cost.cpu().numpy(), want.astype(np.float32))
    o = order.cpu().numpy()
    assert sorted(o.tolist()) == list(range(N >> cl))
    c = want[o]
    span = c.max() - c.min()
    b = np.minimum(((c - c.min()) * (64 / span)).astype(np.int64), 63) if span > 0 else 0 * c
    assert np.all(np.diff(b) >= 0)  # bucket order
    for k in np.unique(b):  # stable inside a bucket
        assert np.all(np.diff(o[b == k]) > 0)
