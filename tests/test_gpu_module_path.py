"""The reference-API module path on the GPU: GridEncoder (live-row batches,
binned embedding backward, the pybind-signature backward), the sigma_net MLP
module on its MFMA kernels, and the whole field through the modules against
the fused field (nerf/field.py) — the path the reference's
nerf/network_grid.py takes on this package (bench.py `module_path`)."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _encoder(gpu, scale=0.5, seed=0):
    from gridencoder import GridEncoder
    torch.manual_seed(seed)
    enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                      log2_hashmap_size=16, desired_resolution=2048, gridtype="tiled").to(gpu)
    with torch.no_grad():
        enc.embeddings.uniform_(-scale, scale)
    return enc


def _positions(n, seed):
    x = np.random.default_rng(seed).random((n, 3), dtype=np.float32) * 2 - 1
    x[:4] = [[-1, -1, -1], [1, 1, 1], [1, -1, 0.5], [0, 0, 0]]
    return x


@pytest.mark.parametrize("amp", [True, False])
def test_grid_encoder_live_rows_vs_oracle(gpu, amp):
    """GridEncoder on a capacity-sized batch carrying a device live-row count
    (the device-count march's samples): rows [0, m) bit-exact against the
    oracle's forward (f16 table under autocast, per-corner f16 rounding),
    rows [m, cap) zero; the embedding gradient of a capacity-sized upstream
    gradient (junk in the dead rows) equals the exact f64 oracle sum over the
    live rows (gridencoder.cu:226-313 arithmetic, f32 tolerance)."""
    enc = _encoder(gpu)
    cap, m = 40000, 33333
    xw = _positions(cap, 3)
    x = T(xw, gpu)
    m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
    setattr(x, "_dfhip_live_rows", m_dev)
    with torch.autocast("cuda", dtype=torch.float16, enabled=amp):
        y = enc(x, bound=1)
    assert y.shape == (cap, 32) and y.dtype == (torch.float16 if amp else torch.float32)
    offs = enc.offsets_host
    S = float(np.log2(enc.per_level_scale))
    x01 = ((T(xw[:m], gpu) + 1) / 2).cpu().numpy()
    emb = enc.embeddings.detach().cpu().numpy()
    want, _ = oracle.grid_encode_forward(x01, emb.astype(np.float16) if amp else emb, offs, S, 16)
    got = y.detach().cpu().numpy()
    np.testing.assert_array_equal(got[:m], want)
    assert not got[m:].any()
    g = np.random.default_rng(4).normal(size=(cap, 32)).astype(np.float32) * 0.1
    g[m:] = 1e3  # dead rows: no gradient may come from them
    gt = T(g.astype(np.float16) if amp else g, gpu)
    y.backward(gt)
    gw = g[:m].astype(np.float16) if amp else g[:m]
    ref = oracle.grid_encode_backward(gw, x01, offs, 2, S, 16)
    got = enc.embeddings.grad.double().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-7 * np.abs(ref).max())


def test_grid_encoder_binned_equals_atomic(gpu):
    """The default binned embedding backward against the reference's atomic
    scatter (GridEncoder.backward_mode = "atomic"), f32 table: the same sum up
    to f32 ordering."""
    grads = []
    xw = _positions(30000, 5)
    g = T(np.random.default_rng(6).normal(size=(30000, 32)).astype(np.float32), gpu)
    for mode in ("binned", "atomic"):
        enc = _encoder(gpu)
        enc.backward_mode = mode
        enc(T(xw, gpu), bound=1).backward(g)
        grads.append(enc.embeddings.grad.double().cpu().numpy())
    np.testing.assert_allclose(grads[0], grads[1], rtol=1e-4, atol=1e-5 * np.abs(grads[1]).max())


@pytest.mark.parametrize("acc", [torch.float32, torch.float16])
def test_pybind_grid_encode_backward_binned(gpu, acc):
    """`_gridencoder.grid_encode_backward` (the reference's pybind signature,
    grad [L, B, C], grad_embeddings zero-filled by the caller and ADDED into)
    now runs the binned walk: against the exact oracle, f32 at f32 tolerance,
    an f16 destination at SURVEY a12's 1e-3 (the reference rounds every f16
    atomic add)."""
    import _gridencoder
    enc = _encoder(gpu)
    offs = enc.offsets_host
    S = float(np.log2(enc.per_level_scale))
    B = 25000
    x01 = (_positions(B, 7) + 1) / 2
    g = (np.random.default_rng(8).normal(size=(16, B, 2)) * 0.1).astype(np.float16)
    emb16 = enc.embeddings.detach().half().contiguous()
    gemb = torch.zeros(int(offs[-1]), 2, dtype=acc, device=gpu)
    gemb += 1.0  # ADDED into: the result is 1 + the gradient
    _gridencoder.grid_encode_backward(T(g, gpu), T(x01, gpu), emb16, enc.offsets, gemb, B, 3, 2,
                                      16, S, 16, None, None, 1, False)
    ref = oracle.grid_encode_backward(g, x01, offs, 2, S, 16, blc=False)
    got = gemb.double().cpu().numpy() - 1.0
    tol = 1e-3 if acc == torch.float16 else 1e-5
    np.testing.assert_allclose(got, ref, rtol=tol, atol=tol * np.abs(ref).max() + 1e-3 * (
        acc == torch.float16))


def _layers(gpu, seed=1):
    torch.manual_seed(seed)
    return [torch.nn.Linear(32, 64).to(gpu), torch.nn.Linear(64, 64).to(gpu),
            torch.nn.Linear(64, 4).to(gpu)]


def _torch_mlp(x, layers):
    h = x
    for i, lin in enumerate(layers):
        h = lin(h)
        if i < 2:
            h = torch.relu(h)
    return h


@pytest.mark.parametrize("elem", [torch.float16, torch.bfloat16])
def test_native_mlp_matches_torch_autocast(gpu, elem):
    """The sigma_net MLP module on dfhip_mlp_forward / _backward against the
    same nn.Linear stack run by torch under autocast: outputs within one
    rounding of the element type, input and weight gradients within the
    activations' rounding (relative norm)."""
    from nerf.mlp import mlp_forward
    layers = _layers(gpu)
    M = 50000
    x = (torch.randn(M, 32, device=gpu) * 0.5).to(elem).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    dh = (torch.randn(M, 4, device=gpu) * 0.1).to(elem)
    with torch.autocast("cuda", dtype=elem):
        h = mlp_forward(x, layers)
        h2 = _torch_mlp(x2, layers)
    assert h.dtype == elem and h2.dtype == elem
    tol = 4e-3 if elem == torch.float16 else 3e-2
    np.testing.assert_allclose(h.float().detach().cpu().numpy(), h2.float().detach().cpu().numpy(),
                               rtol=tol, atol=tol)
    h.backward(dh)
    g_native = [x.grad.float()] + [p.grad.clone() for lin in layers for p in (lin.weight, lin.bias)]
    for lin in layers:
        lin.weight.grad = lin.bias.grad = None
    h2.backward(dh)
    g_torch = [x2.grad.float()] + [p.grad for lin in layers for p in (lin.weight, lin.bias)]
    for a, b in zip(g_native, g_torch):
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < (1e-2 if elem == torch.float16 else 5e-2), rel


def test_native_mlp_live_rows(gpu):
    """Capacity-sized features with a device live-row count: rows past it come
    out zero (output and input gradient), and the weight gradients equal those
    of the live rows alone (junk upstream gradient in the dead rows)."""
    from nerf.mlp import mlp_forward
    layers = _layers(gpu, 2)
    cap, m = 40000, 29999
    base = torch.randn(cap, 32, device=gpu).half()
    m_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
    dh = torch.randn(cap, 4, device=gpu).half()
    dh[m:] = 100.0
    outs = []
    for rows, live in ((cap, m_dev), (m, None)):
        x = base[:rows].clone().requires_grad_(True)
        if live is not None:
            setattr(x, "_dfhip_live_rows", live)
        with torch.autocast("cuda", dtype=torch.float16):
            h = mlp_forward(x, layers)
        h.backward(dh[:rows])
        outs.append((h.detach(), x.grad, [p.grad.clone() for lin in layers
                                          for p in (lin.weight, lin.bias)]))
        for lin in layers:
            lin.weight.grad = lin.bias.grad = None
    (h0, dx0, g0), (h1, dx1, g1) = outs
    assert torch.equal(h0[:m], h1) and not h0[m:].any()
    assert torch.equal(dx0[:m], dx1) and not dx0[m:].any()
    for a, b in zip(g0, g1):  # a different part split: f32 summation order only
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_module_field_matches_fused_field(gpu):
    """network_grid.common_forward through the modules (GridEncoder -> MLP ->
    trunc_exp / sigmoid, fused_field = False) against the fused field node
    (nerf/field.py) on the same samples and upstream gradients: the same
    autocast arithmetic, so sigma / albedo agree to f16 rounding and every
    parameter gradient to the activations' rounding."""
    import main
    from nerf.network_grid import NeRFNetwork
    opt = main.parse_opt(["--text", "x", "-O"])
    torch.manual_seed(0)
    net = NeRFNetwork(opt).to(gpu)
    with torch.no_grad():
        net.encoder.embeddings.uniform_(-0.5, 0.5)
    x = T(_positions(60000, 9) * 0.9, gpu)
    gs = torch.randn(60000, device=gpu) * 1e-3
    ga = torch.randn(60000, 3, device=gpu) * 1e-2
    res = []
    for fused in (True, False):
        net.fused_field = fused
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            sigma, albedo = net.common_forward(x)
        (sigma.float() * gs).sum().backward(retain_graph=True)
        (albedo.float() * ga).sum().backward()
        res.append((sigma.detach().float(), albedo.detach().float(),
                    [p.grad.clone() for p in (net.encoder.embeddings, *net.sigma_net.parameters())]))
    (s0, a0, g0), (s1, a1, g1) = res
    torch.testing.assert_close(s1, s0, rtol=5e-3, atol=1e-4)
    torch.testing.assert_close(a1, a0, rtol=5e-3, atol=2e-3)
    for a, b in zip(g1, g0):
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < 2e-2, rel


def _module_trainer(seed=3, res=64):
    import bench
    tr, data = bench.make_trainer(res, seed, 0, 1, True, graph=True)
    tr.native_step = False
    tr.model.fused_field = False
    return tr, data


def test_bucketed_module_step_rows_do_not_matter(gpu):
    """BucketedModuleStep's body on the exact sample count M and on the padded
    bucket (rows [M, Mb) zero, the device live count on the views): the same
    draws give the same parameter gradients (the dead rows contribute
    nothing; only the MLP weight-gradient part split differs, f32 order)."""
    from nerf.graph import BucketedModuleStep
    tr, data = _module_trainer()
    for i in range(3):  # a few steps: the occupancy grid and samples move
        tr.train_iteration(data.collate([i]))
    g = next(iter(tr._graphs.values()))
    assert isinstance(g, BucketedModuleStep) and g.graphs
    batch = data.collate([5])
    text_z = tr.text_z[batch["dir"]]
    g.text_z = text_z.detach().clone()
    M = g.march(batch)
    Mb = g.bucket(M)
    assert Mb > M
    g.xyzs[M:Mb].zero_()
    g.dirs[M:Mb].zero_()
    g.deltas[M:Mb].zero_()
    grads = []
    for rows in (M, Mb):
        torch.manual_seed(11)
        for p in g.params:  # as at capture: fresh gradients, copied into the bucket views
            p.grad = None
        g._body(rows)
        torch.cuda.synchronize()
        grads.append([v.detach().clone() for v in g.grad_views])
        for p, v in zip(g.params, g.grad_views):
            p.grad = v
    for a, b in zip(*grads):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-7)
    assert any(a.abs().sum() > 0 for a in grads[0])


def test_bucketed_module_training(gpu):
    """Graph-replayed module-path steps: captured per bucket, finite losses,
    the parameters move, every gradient is a view of the flat bucket the
    optimizer steps, step_counter holds every step's count."""
    from nerf.graph import BucketedModuleStep
    tr, data = _module_trainer(seed=4)
    start = [p.detach().clone() for p in tr.model.parameters()]
    losses = [float(tr.train_iteration(data.collate([i % 4]))) for i in range(10)]
    torch.cuda.synchronize()
    g = next(iter(tr._graphs.values()))
    assert isinstance(g, BucketedModuleStep) and len(g.graphs) >= 1
    M, rows = g.last_rows
    assert M <= rows < 1.25 * max(M, g.MIN_ROWS) + g.ALIGN
    assert all(np.isfinite(losses))
    assert int((tr.model.step_counter[:, 0] > 0).sum()) == len(losses)  # one row per step
    moved = [not torch.equal(a, b) for a, b in zip(start, tr.model.parameters())]
    assert all(moved)
    flat = g.grad_bucket
    for p, v in zip(g.params, g.grad_views):
        assert p.grad is v and torch.isfinite(v).all()
    assert flat.abs().sum() > 0
