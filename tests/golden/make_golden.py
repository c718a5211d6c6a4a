"""Generate tests/golden/golden.npz — seeded input/output vectors of the hot
path, computed by the CPU oracle (oracle/oracle.c).

The reference ships no golden vectors for this path and its extensions cannot
be built here, so these fixtures pin the *oracle*: any later
change to the restatement or to the HIP kernels is checked against the same
committed bytes (tests/test_golden.py).  Regenerate only on a deliberate
oracle change:

    python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
sys.path.insert(0, str(HERE.parent))

import oracle  # noqa: E402
from scenes import AABB, camera_rays, sphere_bitfield  # noqa: E402

OUT = HERE / "golden.npz"

# reduced grid-encoder config (same level formula as network_grid.py:49 but
# a 2^10 table so the fixture stays small): L=16, C=2, H=16, desired 256
GRID_L, GRID_C, GRID_H, GRID_LOG2T, GRID_DESIRED = 16, 2, 16, 10, 256


def level_offsets(L, C, D, H, per_level_scale, log2_hashmap):
    """gridencoder/grid.py:110-124 restated."""
    offs, off = [], 0
    max_params = 2 ** log2_hashmap
    for i in range(L):
        res = int(np.ceil(H * per_level_scale ** i))
        p = min(max_params, (res + 1) ** D)
        p = int(np.ceil(p / 8) * 8)
        offs.append(off)
        off += p
    offs.append(off)
    return np.array(offs, np.int32)


def main():
    g = {}
    # ------------------------------------------------------------- march
    rays_o, rays_d = camera_rays(12, 12, seed=3)
    nears, fars = oracle.near_far_from_aabb(rays_o, rays_d, AABB, 0.2)
    noises = np.random.default_rng(7).random(rays_o.shape[0], dtype=np.float32)
    bf = sphere_bitfield(0.5, 0.002, 3)
    counts, xyzs, dirs, deltas = oracle.march_rays_train(rays_o, rays_d, bf, 1.0, 0.0, 512, 1, 128,
                                                         nears, fars, noises)
    g.update(rays_o=rays_o, rays_d=rays_d, nears=nears, fars=fars, noises=noises, bitfield=bf,
             march_counts=counts, march_xyzs=xyzs, march_dirs=dirs, march_deltas=deltas)
    # ------------------------------------------------------------- composite
    r = np.random.default_rng(11)
    m = xyzs.shape[0]
    sig = (r.random(m, dtype=np.float32) * 40).astype(np.float32)
    rgb = r.random((m, 3), dtype=np.float32)
    rays = oracle.rays_from_counts(counts)
    ws, depth, image = oracle.composite_rays_train_forward(sig, rgb, deltas, rays, 1e-4)
    gws = r.standard_normal(rays.shape[0]).astype(np.float32)
    gim = r.standard_normal((rays.shape[0], 3)).astype(np.float32)
    gs, gc = oracle.composite_rays_train_backward(gws, gim, sig, rgb, deltas, rays, ws, image, 1e-4)
    g.update(comp_sigmas=sig, comp_rgbs=rgb, comp_ws=ws, comp_depth=depth, comp_image=image,
             comp_grad_ws=gws, comp_grad_image=gim, comp_grad_sigmas=gs, comp_grad_rgbs=gc)
    # ------------------------------------------------------------- inference march + composite
    n = rays_o.shape[0]
    alive = np.arange(n, dtype=np.int32)
    rays_t = nears.copy()
    inoise = np.random.default_rng(13).random(n, dtype=np.float32)
    ix, idr, idl = oracle.march_rays(n, 4, alive, rays_t, rays_o, rays_d, 1.0, 0.0, 512, 1, 128,
                                     bf, fars, inoise)
    isig = (np.random.default_rng(17).random(n * 4, dtype=np.float32) * 20).astype(np.float32)
    irgb = np.random.default_rng(19).random((n * 4, 3), dtype=np.float32)
    a2, t2 = alive.copy(), rays_t.copy()
    iws, idep, iimg = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
    oracle.composite_rays(n, 4, 1e-4, a2, t2, isig, irgb, idl, iws, idep, iimg)
    g.update(inf_noises=inoise, inf_xyzs=ix, inf_dirs=idr, inf_deltas=idl, inf_sigmas=isig,
             inf_rgbs=irgb, inf_rays_alive=a2, inf_rays_t=t2, inf_ws=iws, inf_depth=idep,
             inf_image=iimg)
    # ------------------------------------------------------------- morton / packbits
    coords = np.random.default_rng(23).integers(0, 128, (4096, 3)).astype(np.int32)
    grid = (np.random.default_rng(29).random((1, 8192), dtype=np.float32) * 2).astype(np.float32)
    g.update(morton_coords=coords, morton_indices=oracle.morton3D(coords), pack_grid=grid,
             pack_bits=oracle.packbits(grid, 1.0))
    # ------------------------------------------------------------- grid encoder
    pls = np.exp2(np.log2(GRID_DESIRED / GRID_H) / (GRID_L - 1))
    S = np.float32(np.log2(pls))
    offs = level_offsets(GRID_L, GRID_C, 3, GRID_H, pls, GRID_LOG2T)
    r = np.random.default_rng(31)
    emb = ((r.random((int(offs[-1]), GRID_C), dtype=np.float32) - 0.5) * 2).astype(np.float32)
    x = r.random((600, 3), dtype=np.float32)
    x[:5] = [[0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.5], [1.0001, 0.2, 0.2], [0.3, -0.01, 0.3]]
    out32, dy = oracle.grid_encode_forward(x, emb, offs, float(S), GRID_H, 1, False, True)
    out16, _ = oracle.grid_encode_forward(x, emb.astype(np.float16), offs, float(S), GRID_H, 1,
                                          False, False)
    outh, _ = oracle.grid_encode_forward(x, emb, offs, float(S), GRID_H, 0, False, False)
    gg = r.standard_normal((600, GRID_L * GRID_C)).astype(np.float32)
    gemb = oracle.grid_encode_backward(gg, x, offs, GRID_C, float(S), GRID_H, 1, False, True)
    g.update(grid_S=np.array(S, np.float32), grid_H=np.array(GRID_H, np.int32), grid_offsets=offs,
             grid_embeddings=emb, grid_inputs=x, grid_out_f32=out32, grid_dy_dx=dy,
             grid_out_f16=out16, grid_out_hash=outh, grid_grad=gg, grid_grad_embeddings=gemb)
    # ------------------------------------------------------------- freq encoder
    fx = ((np.random.default_rng(37).random((200, 3), dtype=np.float32) - 0.5) * 4).astype(np.float32)
    fo = oracle.freq_encode_forward(fx, 6)
    fg = np.random.default_rng(41).standard_normal(fo.shape).astype(np.float32)
    g.update(freq_inputs=fx, freq_out=fo, freq_grad=fg,
             freq_grad_inputs=oracle.freq_encode_backward(fg, fo, 3, 6))
    np.savez_compressed(OUT, **g)
    print(OUT, OUT.stat().st_size, "bytes;", ", ".join(f"{k}{tuple(v.shape)}" for k, v in g.items()))


if __name__ == "__main__":
    main()
