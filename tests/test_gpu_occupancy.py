"""Occupancy-grid refresh (rows a9 / f2: `update_extra_state`, reference
nerf/renderer.py:563-613) on the product path — the fused field forward at
the jittered cell positions, `dfhip_density_grid_ema` and
`dfhip_packbits_mean` (csrc/occupancy.hip), `dfhip_mean_count` — against the
CPU oracle:

* positions: the reference's cell coordinates, morton indices
  (oracle.morton3D) and jitter arithmetic (renderer.py:580-593) restated in
  numpy f32 on the same uniform draws (the refresh's generator replayed);
* sigma: oracle/field.py's field restatement (f16 or bf16 autocast), with
  its propagated rounding windows (the same model as test_gpu_field_oracle);
* EMA-max over valid cells (renderer.py:600-601): every refreshed cell lies in
  [max(decay * old, sigma_lo), max(decay * old, sigma_hi)], cells with
  old < 0 are untouched;
* mean over valid cells (renderer.py:602) against the float64 mean of the
  refreshed grid; the bitfield bit-exact against oracle.packbits at
  min(mean, density_thresh) (renderer.py:606-607, raymarching.cu:265-285);
  mean_count = int(sum / total_step) exactly (renderer.py:610-613).

The oracle sigma is evaluated on a seeded subset of the cells (all cascades)
so the test stays within seconds of CPU time; the bitfield and mean are
checked on every cell.
"""
import numpy as np
import pytest
import torch

import oracle
import oracle.field as of
from test_gpu_field_oracle import MFMA_ULPS

pytestmark = pytest.mark.gpu

F32 = np.float32
SUBSET = 200_000


def _cell_points(G):
    """renderer.py:581-584: meshgrid (ij) coordinates, morton indices and
    2 * c / (G - 1) - 1 in f32.  torch's CUDA true division by a Python scalar
    multiplies by the f32 reciprocal (BinaryDivTrueKernel), so the reference's
    positions are (2 c) * f32(1 / (G - 1)) - 1."""
    ax = np.arange(G, dtype=np.int32)
    xx, yy, zz = np.meshgrid(ax, ax, ax, indexing="ij")
    coords = np.stack([xx.reshape(-1), yy.reshape(-1), zz.reshape(-1)], -1).astype(np.int32)
    idx = oracle.morton3D(coords).astype(np.int64)
    xyz = (F32(2) * coords.astype(F32)) * (F32(1) / F32(G - 1)) - F32(1)
    return xyz.astype(F32), idx


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_grid_refresh_matches_oracle(gpu, dtype):
    import bench
    bf = dtype == torch.bfloat16
    trainer, data = bench.make_trainer(64, 11, 0, 1, True, bf16=bf)
    for i in range(3):
        trainer.train_iteration(data.collate([i % 4]))
    m = trainer.model
    assert m.native_grid_update and m.density_grid.is_cuda
    G, CAS = m.grid_size, m.cascade
    cells = G ** 3
    g = torch.Generator(device=gpu).manual_seed(5)
    with torch.no_grad():
        m.encoder.embeddings.uniform_(-0.5, 0.5, generator=g)
        # old values on the scale of the queried sigmas, so both EMA branches occur
        old = torch.rand(m.density_grid.shape, generator=g, device=gpu) * 2
        old[torch.rand(old.shape, generator=g, device=gpu) < 0.05] = -1.0
        m.density_grid.copy_(old)
    old_np = old.cpu().numpy().astype(F32)
    counts = m.step_counter.cpu().numpy()
    local = m.local_step
    it0 = m.iter_density

    m.grid_generator = torch.Generator(device=gpu).manual_seed(77)
    with torch.autocast("cuda", dtype=dtype):
        m.update_extra_state()
    torch.cuda.synchronize()
    grid = m.density_grid.cpu().numpy()
    bits = m.density_bitfield.cpu().numpy()
    mean = float(m.mean_density)
    assert m.iter_density == it0 + 1 and m.local_step == 0

    # ---- positions (the refresh's draws replayed) and the oracle sigma
    xyz, idx = _cell_points(G)
    pxyz, pidx = m._grid_points()
    assert np.array_equal(pidx.cpu().numpy().astype(np.int64), idx)
    assert np.array_equal(pxyz.cpu().numpy(), xyz), "cell positions differ from the restatement"
    replay = torch.Generator(device=gpu).manual_seed(77)
    enc = m.encoder
    emb = enc.embeddings.detach().float().cpu().numpy()
    offsets = enc.offsets.cpu().numpy()
    S = float(np.log2(enc.per_level_scale))
    Hb = int(enc.base_resolution)
    ws = [p.detach().float().cpu().numpy() for lin in m.sigma_net.net
          for p in (lin.weight, lin.bias)]
    pick = np.random.default_rng(3).choice(cells, SUBSET, replace=False)
    decay = F32(0.95)
    checked = 0
    for cas in range(CAS):
        bound = min(2 ** cas, m.bound)
        half = bound / G
        u = torch.rand((cells, 3), generator=replay, device=gpu).cpu().numpy()
        pts = xyz * F32(bound - half) + (u * F32(2) - F32(1)) * F32(half)
        p = pts[pick]
        with of.precision("bf16" if bf else "f16"):
            f = (of.encode_bf16 if bf else of.encode)(p, m.bound, emb, offsets, S, Hb)
            fo = of.field_forward(p, ws, f)
            fb = of.forward_bounds(fo, ws, acc_ulps=MFMA_ULPS)
        lg = np.log(fo["sigma"].astype(np.float64))
        s_lo, s_hi = np.exp(lg - fb["dlog_sigma"]), np.exp(lg + fb["dlog_sigma"])
        o = old_np[cas, idx[pick]]
        got = grid[cas, idx[pick]].astype(np.float64)
        valid = o >= 0
        od = (o * decay).astype(np.float64)  # f32 product, as torch's
        lo, hi = np.maximum(od, s_lo), np.maximum(od, s_hi)
        v = valid
        bad = (got[v] < lo[v]) | (got[v] > hi[v])
        assert not bad.any(), (
            f"cascade {cas}: {bad.sum()} refreshed cells outside [max(decay*old, sigma_lo), "
            f"max(decay*old, sigma_hi)]")
        assert np.array_equal(got[~v], o[~v].astype(np.float64)), "invalid cells changed"
        checked += int(v.sum())
        print(f"\n[{dtype}] cascade {cas}: {v.sum()} valid cells checked, "
              f"sigma window open on {(fb['dh'][:, 0] > 0).mean():.2e}, "
              f"EMA kept decay*old on {(got[v] == od[v]).mean():.3f}")
    assert checked > SUBSET * CAS * 0.9

    # ---- mean over valid cells, threshold, bitfield, mean_count
    valid_all = old_np >= 0
    want_mean = grid[valid_all].astype(np.float64).mean()
    assert abs(mean - want_mean) <= 1e-6 * abs(want_mean), (mean, want_mean)
    thresh = min(mean, float(m.density_thresh))
    want_bits = oracle.packbits(grid.reshape(-1), thresh)
    assert np.array_equal(bits.reshape(-1), want_bits), \
        f"{int((bits.reshape(-1) != want_bits).sum())} bitfield bytes differ"
    total = min(16, local)
    assert total > 0
    assert int(m.mean_count) == int(counts[:total, 0].astype(np.int64).sum() / total)
