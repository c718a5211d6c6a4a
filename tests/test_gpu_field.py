"""Fused field head (csrc/fieldmlp.hip + nerf/field.py, the product autograd
path) against the CPU oracle of the reference composition (GridEncoder ->
nn.Linear/ReLU stack under fp16 autocast -> trunc_exp(h0 + gaussian) /
sigmoid, network_grid.py:13-32,76-87): oracle/field.py with its propagated
f16-rounding windows (tests/oracle_checks.py), forward and all gradients."""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _field(gpu, seed=0, emb_scale=0.5):
    from gridencoder import GridEncoder
    torch.manual_seed(seed)
    enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                      log2_hashmap_size=16, desired_resolution=2048, gridtype="tiled").to(gpu)
    with torch.no_grad():
        enc.embeddings.uniform_(-emb_scale, emb_scale)
    layers = nn.ModuleList([nn.Linear(32, 64), nn.Linear(64, 64), nn.Linear(64, 4)]).to(gpu)
    return enc, layers


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M", [1, 31, 50_003])
def test_fused_field_matches_oracle(gpu, M, dtype):
    """fp16 autocast (the reference's -O) and bf16 autocast (the C5 option)."""
    from nerf.field import eligible, grid_field
    from oracle_checks import check_field
    enc, layers = _field(gpu)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.rand(M, 3, generator=g) * 2 - 1).mul_(0.9).to(gpu)
    gs = (torch.randn(M, generator=g) * 1e-2).to(gpu)
    ga = (torch.randn(M, 3, generator=g) * 1e-2).to(gpu)
    with torch.autocast("cuda", dtype=dtype):
        assert eligible(enc, layers, x)
        s1, a1 = grid_field(x, 1.0, enc, layers)
    assert s1.dtype == torch.float32 and a1.dtype == dtype
    bf16 = dtype == torch.bfloat16
    ga_np = ga.to(dtype).float().cpu().numpy() if bf16 else ga.cpu().numpy().astype(np.float16)
    params = [enc.embeddings] + list(layers.parameters())
    g1 = torch.autograd.grad((s1 * gs).sum() + (a1.float() * ga).sum(), params)
    for t in g1:
        assert t.dtype == torch.float32
    ws = [p.detach().float().cpu().numpy() for p in layers.parameters()]
    stats = check_field(x.cpu().numpy(), enc.embeddings.detach().cpu().numpy(),
                        enc.offsets.cpu().numpy(), float(np.log2(enc.per_level_scale)), 16, ws,
                        s1.detach().cpu().numpy(), a1.detach().float().cpu().numpy(),
                        gs.cpu().numpy(), ga_np,
                        [t.cpu().numpy() for t in g1[1:]], g1[0].cpu().numpy(),
                        label=f"M={M} {dtype}", bf16=bf16)
    print(stats)


def test_fused_field_deterministic(gpu):
    from nerf.field import grid_field
    enc, layers = _field(gpu, seed=2)
    x = (torch.rand(70_001, 3, device=gpu) * 2 - 1)
    gs = torch.randn(70_001, device=gpu)
    outs = []
    for _ in range(2):
        with torch.autocast("cuda", dtype=torch.float16):
            s, a = grid_field(x, 1.0, enc, layers)
        gr = torch.autograd.grad((s * gs).sum() + a.float().sum(),
                                 [enc.embeddings] + list(layers.parameters()))
        outs.append([s, a] + list(gr))
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def test_fused_field_empty(gpu):
    from nerf.field import grid_field
    enc, layers = _field(gpu)
    x = torch.zeros(0, 3, device=gpu, requires_grad=False)
    with torch.autocast("cuda", dtype=torch.float16):
        s, a = grid_field(x, 1.0, enc, layers)
    assert s.shape == (0,) and a.shape == (0, 3)
    gr = torch.autograd.grad(s.sum() + a.float().sum(), list(layers.parameters()),
                             allow_unused=True)
    for t in gr:
        assert t is None or torch.count_nonzero(t) == 0


def test_fused_field_device_count(gpu):
    """m_dev mode: capacity-sized buffers, live row count read on the device —
    same outputs on the live rows and the same gradients as an exact-size call."""
    from nerf.field import grid_field
    enc, layers = _field(gpu, seed=4)
    M, cap = 40_001, 65_536
    x = torch.rand(cap, 3, device=gpu) * 2 - 1
    gs = torch.randn(cap, device=gpu)
    ga = torch.randn(cap, 3, device=gpu)
    params = [enc.embeddings] + list(layers.parameters())
    m_dev = torch.tensor([M], dtype=torch.int32, device=gpu)
    with torch.autocast("cuda", dtype=torch.float16):
        s_cap, a_cap = grid_field(x, 1.0, enc, layers, m_dev)
        s_m, a_m = grid_field(x[:M].contiguous(), 1.0, enc, layers)
    assert torch.equal(s_cap[:M], s_m) and torch.equal(a_cap[:M], a_m)
    # the dead rows carry garbage; their incoming gradient must not matter
    g_cap = torch.autograd.grad((s_cap[:M] * gs[:M]).sum() + (a_cap[:M].float() * ga[:M]).sum(),
                                params)
    g_m = torch.autograd.grad((s_m * gs[:M]).sum() + (a_m.float() * ga[:M]).sum(), params)
    for u, v in zip(g_cap, g_m):
        torch.testing.assert_close(u, v, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("align,lo,hi,gridtype", [(False, -1.0, 1.0, "tiled"),
                                                  (True, -1.0, 1.0, "tiled"),
                                                  (False, 0.999, 1.0, "tiled"),
                                                  (False, -1.0, 1.0, "hash")])
def test_quad_forward_bit_identical(gpu, dtype, align, lo, hi, gridtype):
    """dfhip_grid_quads + dfhip_grid_field_forward_quads (the native step's
    forward) against the table forward: the cast table equals torch's cast,
    features / sigma / rgb are bit-identical (including the far corner of the
    cube, where corners reach the last rows of dense levels); on a hash grid
    the hashed levels fall back to the table."""
    import _fieldmlp
    from gridencoder import GridEncoder
    enc, layers = _field(gpu, seed=5)
    if gridtype == "hash":
        enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                          log2_hashmap_size=16, desired_resolution=2048, gridtype="hash").to(gpu)
        with torch.no_grad():
            enc.embeddings.uniform_(-0.5, 0.5)
    enc.align_corners = align
    S = float(np.log2(enc.per_level_scale))
    Hb, gt = int(enc.base_resolution), enc.gridtype_id
    ws = [p.detach().float().contiguous() for lin in layers for p in (lin.weight, lin.bias)]
    g = torch.Generator(device=gpu).manual_seed(9)
    M = 40_001
    x = (torch.rand(M, 3, device=gpu, generator=g) * (hi - lo) + lo).contiguous()
    x[:8] = torch.tensor([[1.0, 1.0, 1.0], [-1.0, -1.0, -1.0], [1.0, -1.0, 1.0],
                          [0.0, 0.0, 0.0], [1.0, 0.5, -1.0], [-1.0, 1.0, 1.0],
                          [0.99999, 0.99999, 0.99999], [-0.99999, 1.0, 0.3]], device=gpu)
    emb = enc.embeddings.detach()
    rows = emb.shape[0]
    table = torch.empty(rows, 2, device=gpu, dtype=dtype)
    quads = torch.empty(rows, 4, device=gpu, dtype=torch.int32)
    _fieldmlp.grid_quads(emb, enc.offsets, S, Hb, gt, align, table, quads)
    assert torch.equal(table, emb.to(dtype))
    outs = []
    for q in (None, quads):
        e = torch.empty(M, 32, device=gpu, dtype=dtype)
        s = torch.empty(M, device=gpu)
        a = torch.empty(M, 3, device=gpu, dtype=dtype)
        _fieldmlp.grid_field_forward(x, 1.0, table, enc.offsets, S, Hb, gt, align, ws, e, s, a,
                                     None, quads=q)
        outs.append((e, s, a))
    for u, v in zip(*outs):
        assert torch.equal(u.view(torch.int16) if u.dtype != torch.float32 else u,
                           v.view(torch.int16) if v.dtype != torch.float32 else v)
