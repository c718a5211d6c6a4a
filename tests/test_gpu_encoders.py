"""GPU parity of the grid / frequency / SH encoders against the CPU oracle.

Bit-exact: grid forward in f32 and in f16 (the reference's per-corner half
rounding is emulated by the oracle).  Tolerance: grid backward (atomic
accumulation order is not deterministic; f16 accumulation additionally rounds
every partial sum, exactly like the reference's half2 atomics), dy_dx / input
gradients, frequency and SH encoders.
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _grid_consts():
    from gridencoder.grid import level_offsets
    pls = np.exp2(np.log2(2048 / 16) / 15)
    offs = level_offsets(16, 2, 3, 16, pls, 16, False)
    return offs, float(np.log2(pls)), pls


def _samples(n, seed, edge=True):
    r = np.random.default_rng(seed)
    x = r.random((n, 3), dtype=np.float32)
    if edge:
        x[:8] = [[0, 0, 0], [1, 1, 1], [1, 0, 1], [0.5, 1, 0], [1.0000001, 0.5, 0.5],
                 [-1e-7, 0.2, 0.3], [0.999999, 0.999999, 1e-6], [0.25, 0.5, 0.75]]
    return x


@pytest.mark.parametrize("gridtype", [1, 0])
@pytest.mark.parametrize("dtype", [np.float32, np.float16])
def test_grid_forward_bitexact(gpu, gridtype, dtype):
    import _gridencoder
    offs, S, _ = _grid_consts()
    emb = (np.random.default_rng(1).random((int(offs[-1]), 2)) * 2 - 1).astype(dtype)
    x = _samples(20000, 2)
    out = torch.empty(x.shape[0], 32, dtype=torch.float16 if dtype == np.float16 else torch.float32,
                      device=gpu)
    _gridencoder.grid_encode_forward_blc(T(x, gpu), T(emb, gpu), T(offs, gpu), out, x.shape[0], 3,
                                         2, 16, S, 16, None, gridtype, False)
    want, _ = oracle.grid_encode_forward(x, emb, offs, S, 16, gridtype=gridtype)
    np.testing.assert_array_equal(out.cpu().numpy(), want)
    # reference [L, B, C] layout gives the same values
    out_lbc = torch.empty(16, x.shape[0], 2, dtype=out.dtype, device=gpu)
    _gridencoder.grid_encode_forward(T(x, gpu), T(emb, gpu), T(offs, gpu), out_lbc, x.shape[0], 3,
                                     2, 16, S, 16, None, gridtype, False)
    assert torch.equal(out_lbc.permute(1, 0, 2).reshape(-1, 32), out)


@pytest.mark.parametrize("D,C", [(2, 4), (3, 8), (1, 1), (4, 2), (5, 2)])
def test_grid_forward_other_shapes(gpu, D, C):
    import _gridencoder
    from gridencoder.grid import level_offsets
    L, H = 6, 4
    offs = level_offsets(L, C, D, H, 1.5, 12, True)
    emb = np.random.default_rng(D * 10 + C).normal(size=(int(offs[-1]), C)).astype(np.float32)
    x = np.random.default_rng(5).random((3000, D), dtype=np.float32)
    S = float(np.log2(1.5))
    for gt in (0, 1):
        out = torch.empty(3000, L * C, device=gpu)
        _gridencoder.grid_encode_forward_blc(T(x, gpu), T(emb, gpu), T(offs, gpu), out, 3000, D, C,
                                             L, S, H, None, gt, True)
        want, _ = oracle.grid_encode_forward(x, emb, offs, S, H, gridtype=gt, align_corners=True)
        np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_grid_dy_dx_and_input_grad(gpu):
    import _gridencoder
    offs, S, _ = _grid_consts()
    emb = np.random.default_rng(3).normal(size=(int(offs[-1]), 2)).astype(np.float32)
    x = _samples(4000, 4)
    B = x.shape[0]
    out = torch.empty(B, 32, device=gpu)
    dy = torch.empty(B, 16 * 3 * 2, device=gpu)
    _gridencoder.grid_encode_forward_blc(T(x, gpu), T(emb, gpu), T(offs, gpu), out, B, 3, 2, 16, S,
                                         16, dy, 1, False)
    want, wdy = oracle.grid_encode_forward(x, emb, offs, S, 16, calc_dy_dx=True)
    np.testing.assert_array_equal(dy.cpu().numpy(), wdy)
    g = np.random.default_rng(5).normal(size=(B, 32)).astype(np.float32)
    gemb = torch.zeros(int(offs[-1]), 2, device=gpu)
    gin = torch.empty(B, 3, device=gpu)
    _gridencoder.grid_encode_backward_blc(T(g, gpu), T(x, gpu), T(offs, gpu), gemb, B, 3, 2, 16, S,
                                          16, dy, gin, 1, False)
    np.testing.assert_allclose(gin.cpu().numpy(), oracle.grid_input_backward(g, wdy, 3, 2, 16),
                               rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("acc", ["f32", "f16"])
def test_grid_backward(gpu, acc):
    """Embedding gradient vs the exact float64 oracle.  f32 atomics: only the
    summation order differs.  f16 (reference half2 atomics): each partial sum
    is rounded to half, so the tolerance scales with the half ulp of the
    accumulated magnitude."""
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    x = _samples(30000, 6)
    B = x.shape[0]
    g = (np.random.default_rng(7).normal(size=(B, 32)) * 0.1).astype(np.float16)
    want = oracle.grid_encode_backward(g, x, offs, 2, S, 16)
    gemb = torch.zeros(rows, 2, dtype=torch.float32 if acc == "f32" else torch.float16, device=gpu)
    _gridencoder.grid_encode_backward_blc(T(g, gpu), T(x, gpu), T(offs, gpu), gemb, B, 3, 2, 16, S,
                                          16, None, None, 1, False)
    got = gemb.double().cpu().numpy()
    scale = np.abs(want).max()
    if acc == "f32":
        np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-6 * scale)
    else:
        # rows only touched a few times are near exact; the heavily shared
        # coarse rows carry the half rounding of their running sums
        err = np.abs(got - want)
        assert err.max() <= 4e-3 * scale + 1e-3
        fine = slice(int(offs[9]) * 1, rows)
        np.testing.assert_allclose(got[fine], want[fine], rtol=2e-2, atol=2e-3 * scale)
    # reference-form entry point: [L, B, C] grad in the table's dtype
    gl = torch.zeros_like(gemb)
    glbc = T(g, gpu).to(gemb.dtype).view(B, 16, 2).permute(1, 0, 2).contiguous()
    _gridencoder.grid_encode_backward(glbc, T(x, gpu), gemb, T(offs, gpu), gl, B, 3, 2, 16, S, 16,
                                      None, None, 1, False)
    err = np.abs(gl.double().cpu().numpy() - want)
    assert err.max() <= (1e-4 if acc == "f32" else 4e-3) * scale + (0 if acc == "f32" else 1e-3)


@pytest.mark.parametrize("parts", [1, 3, 0])
@pytest.mark.parametrize("out", ["f32", "f16"])
def test_grid_backward_sliced(gpu, parts, out):
    """LDS-sliced backward: f32 sums, so it matches the exact oracle to f32
    rounding (f16 output: one final rounding)."""
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    x = _samples(40000, 16)
    B = x.shape[0]
    g = (np.random.default_rng(17).normal(size=(B, 32)) * 0.1).astype(np.float16)
    want = oracle.grid_encode_backward(g, x, offs, 2, S, 16)
    glbc = T(g, gpu).view(B, 16, 2).transpose(0, 1).contiguous()
    parts = parts or _gridencoder.grid_backward_default_parts(rows, 2)
    partial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, 2, parts), device=gpu)
    dt = torch.float32 if out == "f32" else torch.float16
    gemb = torch.full((rows, 2), float("nan"), dtype=dt, device=gpu)  # overwritten
    _gridencoder.grid_encode_backward_sliced(glbc, T(x, gpu), T(offs, gpu), gemb, rows, B, 3, 2, 16,
                                             S, 16, 1, False, partial, parts)
    got = gemb.double().cpu().numpy()
    scale = np.abs(want).max()
    tol = 1e-6 * scale if out == "f32" else 0
    np.testing.assert_allclose(got, want, rtol=1e-5 if out == "f32" else 1e-3, atol=tol + 1e-7)
    # accumulate mode adds onto the existing buffer
    _gridencoder.grid_encode_backward_sliced(glbc, T(x, gpu), T(offs, gpu), gemb, rows, B, 3, 2, 16,
                                             S, 16, 1, False, partial, parts, accumulate=True)
    np.testing.assert_allclose(gemb.double().cpu().numpy(), 2 * want,
                               rtol=1e-5 if out == "f32" else 2e-3, atol=2 * tol + 1e-7)


@pytest.mark.parametrize("D,C,gt", [(2, 4, 1), (3, 8, 0), (1, 1, 1), (4, 2, 0), (3, 2, 0)])
def test_grid_backward_sliced_shapes(gpu, D, C, gt):
    import _gridencoder
    from gridencoder.grid import level_offsets
    L, H = 8, 4
    offs = level_offsets(L, C, D, H, 2.0, 17, False)
    rows = int(offs[-1])
    x = np.random.default_rng(D + C).random((6000, D), dtype=np.float32)
    g = np.random.default_rng(C).normal(size=(L, 6000, C)).astype(np.float32)
    S = 1.0
    want = oracle.grid_encode_backward(g, x, offs, C, S, H, gridtype=gt, blc=False)
    parts = 2
    partial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, C, parts), device=gpu)
    gemb = torch.empty(rows, C, device=gpu)
    _gridencoder.grid_encode_backward_sliced(T(g, gpu), T(x, gpu), T(offs, gpu), gemb, rows, 6000,
                                             D, C, L, S, H, gt, False, partial, parts)
    np.testing.assert_allclose(gemb.double().cpu().numpy(), want, rtol=1e-5,
                               atol=1e-6 * np.abs(want).max())


def test_grid_backward_sliced_empty_batch(gpu):
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    partial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, 2, 2), device=gpu)
    gemb = torch.full((rows, 2), 5.0, device=gpu)
    e = torch.zeros(16, 0, 2, dtype=torch.float16, device=gpu)
    _gridencoder.grid_encode_backward_sliced(e, torch.zeros(0, 3, device=gpu), T(offs, gpu), gemb,
                                             rows, 0, 3, 2, 16, S, 16, 1, False, partial, 2)
    assert torch.all(gemb == 0)


@pytest.mark.parametrize("dtype,C,B", [(torch.float16, 2, 70001), (torch.float32, 2, 300),
                                       (torch.float32, 1, 257), (torch.float16, 8, 1000),
                                       (torch.float64, 2, 513), (torch.float16, 1, 0)])
def test_grid_grad_blc_to_lbc(gpu, dtype, C, B):
    """Native [B, L*C] -> [L, B, C] copy equals the reference's permute (grid.py:70)."""
    import _gridencoder
    L = 16
    g = torch.randn(B, L * C, device=gpu).to(dtype)
    out = torch.empty(L, B, C, dtype=dtype, device=gpu)
    _gridencoder.grid_grad_blc_to_lbc(g, out, B, L, C)
    assert torch.equal(out, g.view(B, L, C).transpose(0, 1))


def test_grid_backward_hash(gpu):
    import _gridencoder
    offs, S, _ = _grid_consts()
    x = _samples(5000, 8)
    g = np.random.default_rng(9).normal(size=(5000, 32)).astype(np.float32)
    gemb = torch.zeros(int(offs[-1]), 2, device=gpu)
    _gridencoder.grid_encode_backward_blc(T(g, gpu), T(x, gpu), T(offs, gpu), gemb, 5000, 3, 2, 16,
                                          S, 16, None, None, 0, False)
    want = oracle.grid_encode_backward(g, x, offs, 2, S, 16, gridtype=0)
    np.testing.assert_allclose(gemb.double().cpu().numpy(), want, rtol=1e-4,
                               atol=1e-5 * np.abs(want).max())


def test_grid_encoder_module_autocast(gpu):
    """GridEncoder under autocast: half table, [B, 32] half output, f32 grad."""
    from gridencoder import GridEncoder
    enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                      log2_hashmap_size=16, desired_resolution=2048, gridtype="tiled").to(gpu)
    with torch.no_grad():
        enc.embeddings.uniform_(-0.5, 0.5)
    xw = np.random.default_rng(10).random((8000, 3), dtype=np.float32) * 2 - 1
    with torch.autocast("cuda", dtype=torch.float16):
        y = enc(T(xw, gpu), bound=1)
    assert y.dtype == torch.float16 and y.shape == (8000, 32)
    offs = enc.offsets.cpu().numpy()
    S = float(np.log2(enc.per_level_scale))
    emb16 = enc.embeddings.detach().half().cpu().numpy()
    xin = ((T(xw, gpu) + 1) / 2).cpu().numpy()
    want, _ = oracle.grid_encode_forward(xin, emb16, offs, S, 16)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), want)
    y.float().pow(2).sum().backward()
    assert enc.embeddings.grad.dtype == torch.float32
    wg = oracle.grid_encode_backward((2 * y.detach().float()).half().cpu().numpy(), xin, offs, 2, S, 16)
    got = enc.embeddings.grad.double().cpu().numpy()
    assert np.abs(got - wg).max() <= 5e-3 * np.abs(wg).max() + 1e-3


# ------------------------------------------------------------------ freq / sh

def test_freq_encoder(gpu):
    from freqencoder import FreqEncoder
    enc = FreqEncoder(input_dim=3, degree=6)
    x = (np.random.default_rng(11).random((20000, 3)) * 2 - 1).astype(np.float32)
    xt = T(x, gpu).requires_grad_(True)
    y = enc(xt)
    want = oracle.freq_encode_forward(x, 6)
    np.testing.assert_allclose(y.detach().cpu().numpy(), want, rtol=0, atol=2e-6)
    g = np.random.default_rng(12).normal(size=want.shape).astype(np.float32)
    (y * T(g, gpu)).sum().backward()
    gi = oracle.freq_encode_backward(g, y.detach().cpu().numpy(), 3, 6)
    np.testing.assert_allclose(xt.grad.cpu().numpy(), gi, rtol=1e-5, atol=1e-5)


def test_freq_encoder_empty(gpu):
    from freqencoder import FreqEncoder
    y = FreqEncoder(3, 6)(torch.zeros(0, 3, device=gpu))
    assert y.shape == (0, 39)


@pytest.mark.parametrize("degree", [1, 4, 8])
def test_sh_encoder(gpu, degree):
    from shencoder import SHEncoder
    enc = SHEncoder(input_dim=3, degree=degree)
    x = np.random.default_rng(13).normal(size=(5000, 3)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    xt = T(x, gpu).requires_grad_(True)
    y = enc(xt)
    want, jac = oracle.sh_encode(x.astype(np.float64), degree)
    np.testing.assert_allclose(y.detach().cpu().numpy(), want, rtol=1e-5, atol=2e-6)
    g = np.random.default_rng(14).normal(size=want.shape)
    (y * T(g.astype(np.float32), gpu)).sum().backward()
    np.testing.assert_allclose(xt.grad.cpu().numpy(), np.einsum("bk,bdk->bd", g, jac), rtol=1e-4,
                               atol=1e-4)


def _binned(glbc, x, bound, offs, rows, B, m_dev, D, C, L, S, H, gt, gpu, accumulate=False,
            gemb=None, opts=None):
    import _gridencoder
    ne, nc, npf = _gridencoder.grid_backward_binned_scratch(B, offs, L, C, opts)
    ent = torch.empty(ne, dtype=torch.int32, device=gpu)
    cnt = torch.empty(nc, dtype=torch.int32, device=gpu)
    part = torch.full((npf,), float("nan"), device=gpu)
    if gemb is None:
        gemb = torch.full((rows, C), float("nan"), device=gpu)  # overwritten
    _gridencoder.grid_encode_backward_binned(glbc, x, bound, T(offs, gpu), offs, gemb, B, m_dev,
                                             D, C, L, S, H, gt, False, ent, cnt, part,
                                             accumulate, opts=opts)
    return gemb


@pytest.mark.parametrize("gt", [1, 0])
def test_grid_backward_binned(gpu, gt):
    """Binned owner-computes backward (csrc/gridbin.hip) against the exact
    f64 oracle: f64 sums rounded to f32 once."""
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    x = _samples(50000, 21)
    B = x.shape[0]
    g = (np.random.default_rng(22).normal(size=(B, 32)) * 0.1).astype(np.float16)
    want = oracle.grid_encode_backward(g, x, offs, 2, S, 16, gridtype=gt)
    glbc = T(g, gpu).view(B, 16, 2).transpose(0, 1).contiguous()
    gemb = _binned(glbc, T(x, gpu), 0.0, offs, rows, B, None, 3, 2, 16, S, 16, gt, gpu)
    scale = np.abs(want).max()
    np.testing.assert_allclose(gemb.double().cpu().numpy(), want, rtol=1e-6, atol=1e-7 * scale)
    _binned(glbc, T(x, gpu), 0.0, offs, rows, B, None, 3, 2, 16, S, 16, gt, gpu,
            accumulate=True, gemb=gemb)
    np.testing.assert_allclose(gemb.double().cpu().numpy(), 2 * want, rtol=1e-6,
                               atol=2e-7 * scale)


def test_grid_backward_binned_device_count(gpu):
    """Capacity-sized planes, live count on the device, raw [-bound, bound]
    positions: only rows [0, m) contribute (the graph-captured train step)."""
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    cap, m, bound = 9000, 6123, 1.0
    x01 = _samples(cap, 23, edge=False)
    g = (np.random.default_rng(24).normal(size=(cap, 32)) * 0.1).astype(np.float16)
    want = oracle.grid_encode_backward(g[:m], x01[:m], offs, 2, S, 16)
    glbc = T(g, gpu).view(cap, 16, 2).transpose(0, 1).contiguous()
    xr = T(x01 * 2 * bound - bound, gpu)
    m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
    gemb = _binned(glbc, xr, bound, offs, rows, cap, m_dev, 3, 2, 16, S, 16, 1, gpu)
    scale = np.abs(want).max()
    np.testing.assert_allclose(gemb.double().cpu().numpy(), want, rtol=1e-5, atol=1e-6 * scale)


@pytest.mark.parametrize("C,L,H,log2T", [(1, 8, 4, 17), (4, 6, 8, 15), (2, 16, 16, 19),
                                         (2, 20, 4, 14), (2, 24, 2, 12)])
def test_grid_backward_binned_shapes(gpu, C, L, H, log2T):
    """Other layouts, including C = 2 with more than 16 levels (the row ->
    level search of k_sum2 reaches every level, not only the first 16)."""
    from gridencoder.grid import level_offsets
    offs = level_offsets(L, C, 3, H, 2.0, log2T, False)
    rows = int(offs[-1])
    x = np.random.default_rng(C + L).random((7000, 3), dtype=np.float32)
    g = np.random.default_rng(C).normal(size=(L, 7000, C)).astype(np.float32)
    want = oracle.grid_encode_backward(g, x, offs, C, 1.0, H, gridtype=1, blc=False)
    gemb = _binned(T(g, gpu), T(x, gpu), 0.0, offs, rows, 7000, None, 3, C, L, 1.0, H, 1, gpu)
    np.testing.assert_allclose(gemb.double().cpu().numpy(), want, rtol=1e-5,
                               atol=1e-6 * np.abs(want).max())


def test_grid_backward_binned_empty(gpu):
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    m_dev = torch.zeros(1, dtype=torch.int32, device=gpu)
    e = torch.zeros(16, 100, 2, dtype=torch.float16, device=gpu)
    gemb = _binned(e, torch.zeros(100, 3, device=gpu), 1.0, offs, rows, 100, m_dev, 3, 2, 16, S,
                   16, 1, gpu)
    assert torch.all(gemb == 0)


def test_grid_backward_binned_phases(gpu):
    """The phase-split entry point: bin (phase 1) then walk + sum (phase 2),
    as two launches, equals the one-call form (phase 3) bit for bit."""
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    x = T(_samples(30000, 31), gpu)
    B = x.shape[0]
    g = (np.random.default_rng(32).normal(size=(B, 32)) * 0.1).astype(np.float16)
    glbc = T(g, gpu).view(B, 16, 2).transpose(0, 1).contiguous()
    ne, nc, npf = _gridencoder.grid_backward_binned_scratch(B, offs, 16, 2)
    out = {}
    for mode in ("split", "whole"):
        ent = torch.empty(ne, dtype=torch.int32, device=gpu)
        cnt = torch.empty(nc, dtype=torch.int32, device=gpu)
        part = torch.full((npf,), float("nan"), device=gpu)
        gemb = torch.full((rows, 2), float("nan"), device=gpu)
        args = (glbc, x, 0.0, T(offs, gpu), offs, gemb, B, None, 3, 2, 16, S, 16, 1, False, ent,
                cnt, part)
        if mode == "split":
            _gridencoder.binned_launcher(*args, phase=1)()
            _gridencoder.binned_launcher(*args, phase=2)()
        else:
            _gridencoder.binned_launcher(*args, phase=3)()
        out[mode] = gemb
    torch.cuda.synchronize()
    assert torch.isfinite(out["whole"]).all()
    assert torch.equal(out["split"], out["whole"])
    with pytest.raises(RuntimeError):
        _gridencoder.binned_launcher(*args, phase=4)


@pytest.mark.parametrize("gt", [1, 0])
def test_grid_backward_fast_bins_equal_generic(gpu, gt):
    """The mask-form binning fast path (gridbin.hip k_bin_fast: host-evaluated
    level constants, corner slices from x-neighbour pairs) files exactly the
    generic k_bin's entries: same per-(tile, slice) counts, same id set in
    every segment; tiled grid (fast path) and hashed grid (falls back)."""
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    # include points on slice and level edges: lattice-aligned and clamped ones
    x = _samples(40000, 41)
    x[:64] = np.float32(1.0)
    x[64:128] = np.float32(0.0)
    B = x.shape[0]
    g = (np.random.default_rng(42).normal(size=(B, 32)) * 0.1).astype(np.float16)
    glbc = T(g, gpu).view(B, 16, 2).transpose(0, 1).contiguous()
    xt = T(x, gpu)
    ne, nc, npf = _gridencoder.grid_backward_binned_scratch(B, offs, 16, 2)
    got = {}
    for fast in (0, 1):
        opts = _gridencoder.BinnedOpts(fast_bin=fast)
        ent = torch.zeros(ne, dtype=torch.int32, device=gpu)
        cnt = torch.zeros(nc, dtype=torch.int32, device=gpu)
        part = torch.empty(npf, device=gpu)
        gemb = torch.empty(rows, 2, device=gpu)
        _gridencoder.binned_launcher(glbc, xt, 0.0, T(offs, gpu), offs, gemb, B, None, 3, 2,
                                     16, S, 16, gt, False, ent, cnt, part, opts=opts)()
        torch.cuda.synchronize()
        got[fast] = (ent.cpu().numpy().view(np.uint16), cnt.cpu().numpy(), gemb.cpu().numpy())
    tsz = _gridencoder.grid_backward_binned_tile()
    tiles = -(-B // tsz)
    (e0, c0, g0), (e1, c1, g1) = got[0], got[1]
    # counts region [tiles][bins]; bins = slices of 8,192 rows per level (C = 2)
    nb = int(sum(-(-int(offs[l + 1] - offs[l]) // 8192) for l in range(16)))
    assert np.array_equal(c0[:tiles * nb], c1[:tiles * nb])
    assert c0[:tiles * nb].sum() > 16 * (B - 128)  # every in-range sample, every level
    for t in range(tiles):
        for b in range(nb):
            n = int(c0[t * nb + b])
            base = (t * nb + b) * tsz
            assert np.array_equal(np.sort(e0[base:base + n]), np.sort(e1[base:base + n])), (t, b)
    np.testing.assert_allclose(g1, g0, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_grid_backward_stencil_groups_equal_rows(gpu, dtype):
    """dfhip_grid_encode_backward_binned_stencil (7-point finite-difference
    groups binned and walked per sample, the shaded train step) equals the
    row-wise binned backward over the 7 M stencil rows laid out by
    dfhip_shading_stencil, and the exact f64 oracle over those rows; device
    count, raw [-1, 1] positions, samples on the box faces (clamped
    stencil points)."""
    import _dfhip
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    cap, m, eps = 6000, 5321, 1e-2
    x = (_samples(cap, 51, edge=False) * 2 - 1).astype(np.float32)
    x[:50, 0] = np.float32(1.0)   # on the +x face: the +x stencil point clamps
    x[50:100, 2] = np.float32(-1.0)
    xt = T(x, gpu)
    m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
    x7 = torch.empty(7 * cap, 3, device=gpu)
    m7 = torch.zeros(1, dtype=torch.int32, device=gpu)
    _dfhip.call("dfhip_shading_stencil", xt.data_ptr(), m_dev.data_ptr(), cap, eps, 1.0,
                x7.data_ptr(), m7.data_ptr(), _dfhip.stream())
    g = (torch.randn(16, 7 * cap, 2, generator=torch.Generator().manual_seed(52)) * 0.1)
    g = g.to(dtype).to(gpu)
    out = {}
    for mode in ("rows", "groups"):
        ne, nc, npf = _gridencoder.grid_backward_binned_scratch(
            7 * cap if mode == "rows" else cap, offs, 16, 2, group=1 if mode == "rows" else 7)
        ent = torch.empty(ne, dtype=torch.int32, device=gpu)
        cnt = torch.empty(nc, dtype=torch.int32, device=gpu)
        part = torch.empty(npf, device=gpu)
        gemb = torch.full((rows, 2), float("nan"), device=gpu)
        if mode == "rows":
            _gridencoder.binned_launcher(g, x7, 1.0, T(offs, gpu), offs, gemb, 7 * cap, m7, 3, 2,
                                         16, S, 16, 1, False, ent, cnt, part)()
        else:
            _gridencoder.binned_launcher(g, xt, 1.0, T(offs, gpu), offs, gemb, cap, m_dev, 3, 2,
                                         16, S, 16, 1, False, ent, cnt, part, stencil_eps=eps)()
        torch.cuda.synchronize()
        out[mode] = gemb.double().cpu().numpy()
    x01 = ((x7[:7 * m].cpu().numpy() + np.float32(1)) / np.float32(2)).astype(np.float32)
    gl = g[:, :7 * m].float().cpu().numpy()  # [L, 7m, C]
    want = oracle.grid_encode_backward(gl, x01, offs, 2, S, 16, gridtype=1, blc=False)
    scale = np.abs(want).max()
    # the walk's part images are f32: a different split of a slice's entries
    # into parts rounds differently (a few f32 ulps of the parts' magnitude)
    np.testing.assert_allclose(out["groups"], out["rows"], rtol=1e-5, atol=1e-7 * scale)
    np.testing.assert_allclose(out["groups"], want, rtol=1e-5, atol=1e-7 * scale)


def test_binned_options_are_per_call(gpu):
    """dfhip_binned_opts is a per-call argument: a call with debug options (a
    walk trace, the generic binning, 5 walk workgroups per CU) leaves the
    next default call unaffected — no trace written, the default scratch
    size, and the default call's result equal to a default call made before
    any debug call (re-entrant, no global mutable state)."""
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    x = _samples(20000, 71)
    B = x.shape[0]
    g = (np.random.default_rng(72).normal(size=(B, 32)) * 0.1).astype(np.float16)
    glbc = T(g, gpu).view(B, 16, 2).transpose(0, 1).contiguous()
    xt = T(x, gpu)
    scratch0 = _gridencoder.grid_backward_binned_scratch(B, offs, 16, 2)

    def run(opts=None, trace=None):
        ne, nc, npf = _gridencoder.grid_backward_binned_scratch(B, offs, 16, 2, opts)
        ent = torch.zeros(ne, dtype=torch.int32, device=gpu)
        cnt = torch.zeros(nc, dtype=torch.int32, device=gpu)
        part = torch.zeros(npf, device=gpu)
        gemb = torch.empty(rows, 2, device=gpu)
        _gridencoder.binned_launcher(glbc, xt, 0.0, T(offs, gpu), offs, gemb, B, None, 3, 2, 16,
                                     S, 16, 1, False, ent, cnt, part, opts=opts)()
        torch.cuda.synchronize()
        return gemb.cpu().numpy()

    before = run()
    trace = torch.zeros(8 * 16 * 256 * 8, dtype=torch.int64, device=gpu)
    dbg = _gridencoder.BinnedOpts(walk_mode=0, fast_bin=0, walk_groups_per_cu=5, trace=trace)
    assert _gridencoder.grid_backward_binned_scratch(B, offs, 16, 2, dbg)[2] > scratch0[2]
    got_dbg = run(dbg)
    assert int(trace.count_nonzero()) > 0  # the debug call wrote its walk timeline
    trace.zero_()
    after = run()
    torch.cuda.synchronize()
    assert int(trace.count_nonzero()) == 0  # the default call wrote none
    assert _gridencoder.grid_backward_binned_scratch(B, offs, 16, 2) == scratch0
    # same plan and walk: the default result is reproduced (f64 sums of exact
    # products; the debug call's different part split rounds at f32 only)
    np.testing.assert_allclose(after, before, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(got_dbg, before, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("mode", [0, 1])
def test_grid_backward_walk_forms(gpu, mode):
    """Both shipped walk forms of the binned backward (gridbin.hip: 0 = one
    wave per tile segment, 1 = the part's segments end to end in equal runs)
    against the exact f64 oracle, for
    single samples (the albedo step, with a device count and raw positions)
    and for 7-point stencil groups (the shaded steps, samples on the box
    faces)."""
    import _dfhip
    import _gridencoder
    opts = _gridencoder.BinnedOpts(walk_mode=mode)
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    # single samples: capacity planes, live count on the device
    cap, m = 40000, 33333
    x01 = _samples(cap, 61, edge=False)
    g = (np.random.default_rng(62).normal(size=(cap, 32)) * 0.1).astype(np.float16)
    want = oracle.grid_encode_backward(g[:m], x01[:m], offs, 2, S, 16)
    glbc = T(g, gpu).view(cap, 16, 2).transpose(0, 1).contiguous()
    m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
    gemb = _binned(glbc, T(x01 * 2 - 1, gpu), 1.0, offs, rows, cap, m_dev, 3, 2, 16, S, 16,
                   1, gpu, opts=opts)
    scale = np.abs(want).max()
    np.testing.assert_allclose(gemb.double().cpu().numpy(), want, rtol=1e-5,
                               atol=1e-7 * scale)
    # stencil groups
    cap, m, eps = 5000, 4321, 1e-2
    x = (_samples(cap, 63, edge=False) * 2 - 1).astype(np.float32)
    x[:40, 1] = np.float32(1.0)
    xt = T(x, gpu)
    m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
    x7 = torch.empty(7 * cap, 3, device=gpu)
    m7 = torch.zeros(1, dtype=torch.int32, device=gpu)
    _dfhip.call("dfhip_shading_stencil", xt.data_ptr(), m_dev.data_ptr(), cap, eps, 1.0,
                x7.data_ptr(), m7.data_ptr(), _dfhip.stream())
    g7 = (torch.randn(16, 7 * cap, 2, generator=torch.Generator().manual_seed(64)) * 0.1)
    g7 = g7.half().to(gpu)
    ne, nc, npf = _gridencoder.grid_backward_binned_scratch(cap, offs, 16, 2, opts, group=7)
    ent = torch.empty(ne, dtype=torch.int32, device=gpu)
    cnt = torch.empty(nc, dtype=torch.int32, device=gpu)
    part = torch.empty(npf, device=gpu)
    gemb = torch.full((rows, 2), float("nan"), device=gpu)
    _gridencoder.binned_launcher(g7, xt, 1.0, T(offs, gpu), offs, gemb, cap, m_dev, 3, 2, 16,
                                 S, 16, 1, False, ent, cnt, part, stencil_eps=eps,
                                 opts=opts)()
    torch.cuda.synchronize()
    x01 = ((x7[:7 * m].cpu().numpy() + np.float32(1)) / np.float32(2)).astype(np.float32)
    gl = g7[:, :7 * m].float().cpu().numpy()
    want = oracle.grid_encode_backward(gl, x01, offs, 2, S, 16, gridtype=1, blc=False)
    np.testing.assert_allclose(gemb.double().cpu().numpy(), want, rtol=1e-5,
                               atol=1e-7 * np.abs(want).max())


def test_grid_backward_kept_clean_scratch(gpu):
    """BinnedOpts.kept_clean (no clearing launch; the native step's form):
    a run of calls on ONE counts scratch of one capacity B, zeroed once —
    changing live counts (down to zero), a phase-split call and a default
    call in between — equals fresh-scratch default calls bit for bit, and the
    bin totals are zero after every call; the same for stencil groups."""
    import _gridencoder
    offs, S, _ = _grid_consts()
    rows = int(offs[-1])
    tsz = _gridencoder.grid_backward_binned_tile()
    nb = int(sum(-(-int(offs[l + 1] - offs[l]) // 8192) for l in range(16)))
    clean = _gridencoder.BinnedOpts(kept_clean=1)
    for group, cap, seq in ((1, 30000, ((30000, clean, (3,)), (12345, clean, (3,)),
                                        (0, clean, (3,)), (29993, clean, (1, 2)),
                                        (20000, None, (3,)), (29999, clean, (3,)))),
                            (7, 4000, ((4000, clean, (3,)), (1234, clean, (1, 2)),
                                       (0, clean, (3,)), (3999, clean, (3,))))):
        x01 = _samples(cap, 71 + group, edge=False)
        xr = T(x01 * 2 - 1, gpu)
        g = (np.random.default_rng(72).normal(size=(group * cap, 32)) * 0.1).astype(np.float16)
        glbc = T(g, gpu).view(group * cap, 16, 2).transpose(0, 1).contiguous()
        ne, nc, npf = _gridencoder.grid_backward_binned_scratch(cap, offs, 16, 2, group=group)
        scratch = (torch.empty(ne, dtype=torch.int32, device=gpu),
                   torch.zeros(nc, dtype=torch.int32, device=gpu), torch.empty(npf, device=gpu))
        kw = {} if group == 1 else {"stencil_eps": 1e-2}

        def call(m, opts, phases, sc):
            m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
            out = torch.empty(rows, 2, device=gpu)
            for ph in phases:
                _gridencoder.binned_launcher(glbc, xr, 1.0, T(offs, gpu), offs, out, cap, m_dev,
                                             3, 2, 16, S, 16, 1, False, *sc, phase=ph,
                                             opts=opts, **kw)()
            torch.cuda.synchronize()
            return out.cpu().numpy()

        tiles = -(-cap // tsz)
        for m, opts, phases in seq:
            got = call(m, opts, phases, scratch)
            fresh = (torch.empty(ne, dtype=torch.int32, device=gpu),
                     torch.empty(nc, dtype=torch.int32, device=gpu).fill_(-1),
                     torch.empty(npf, device=gpu))
            assert np.array_equal(got, call(m, None, (3,), fresh)), (group, m, phases)
            totals = scratch[1][tiles * nb:tiles * nb + nb * 16]
            assert int(totals.abs().sum()) == 0, (group, m, phases)
