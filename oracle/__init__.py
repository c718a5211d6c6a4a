"""CPU oracle of the reference's NeRF hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the timed CPU baseline; the product
path (single-stable-dreamfusion_amd/) never imports it.

* liboracle.so (oracle.c): scalar C restatement of raymarching.cu,
  gridencoder.cu and freqencoder.cu, exposed here with numpy in/out.
* sh_encode (below): float64 restatement of shencoder.cu's polynomials.
* cpu_render.py: pure-PyTorch CPU restatement of NeRFRenderer.run() + the grid
  network (the reference's --cuda_ray-off path), used as the CPU baseline.

Parity status: UNPINNED against the reference itself (no reference fixtures
exist; building/importing the reference was refused).  The
oracle is pinned by the analytic known-answer tests in tests/test_oracle_kat.py.
"""
from __future__ import annotations

import ctypes
import math
import subprocess
from fractions import Fraction
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists() or LIB.stat().st_mtime < (HERE / "oracle.c").stat().st_mtime:
            build()
        _lib = ctypes.CDLL(str(LIB))
        _lib.orc_march_rays_train.restype = ctypes.c_uint64
        _lib.orc_round_half.restype = ctypes.c_float
        _lib.orc_round_half.argtypes = [ctypes.c_float]
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


_u32 = ctypes.c_uint32
_f = ctypes.c_float


# ---------------------------------------------------------------- raymarching

def near_far_from_aabb(rays_o, rays_d, aabb, min_near=0.2):
    o, d, bb = _f32(rays_o).reshape(-1, 3), _f32(rays_d).reshape(-1, 3), _f32(aabb)
    n = o.shape[0]
    nears, fars = np.empty(n, np.float32), np.empty(n, np.float32)
    lib().orc_near_far_from_aabb(_p(o), _p(d), _p(bb), _u32(n), _f(min_near), _p(nears), _p(fars))
    return nears, fars


def sph_from_ray(rays_o, rays_d, radius):
    o, d = _f32(rays_o).reshape(-1, 3), _f32(rays_d).reshape(-1, 3)
    out = np.empty((o.shape[0], 2), np.float32)
    lib().orc_sph_from_ray(_p(o), _p(d), _f(radius), _u32(o.shape[0]), _p(out))
    return out


def morton3D(coords):
    c = _i32(coords).reshape(-1, 3)
    out = np.empty(c.shape[0], np.int32)
    lib().orc_morton3D(_p(c), _u32(c.shape[0]), _p(out))
    return out


def morton3D_invert(indices):
    i = _i32(indices).reshape(-1)
    out = np.empty((i.shape[0], 3), np.int32)
    lib().orc_morton3D_invert(_p(i), _u32(i.shape[0]), _p(out))
    return out


def packbits(grid, thresh):
    g = _f32(grid)
    n = g.size // 8
    out = np.empty(n, np.uint8)
    lib().orc_packbits(_p(g), _u32(n), _f(thresh), _p(out))
    return out


def march_rays_train(rays_o, rays_d, bitfield, bound, dt_gamma, max_steps, C, H, nears, fars,
                     noises):
    """Per-ray counts and the ray-ordered, contiguous samples.
    Returns counts [N] int32, xyzs [M,3], dirs [M,3], deltas [M,2]."""
    o, d = _f32(rays_o).reshape(-1, 3), _f32(rays_d).reshape(-1, 3)
    bf = np.ascontiguousarray(bitfield, dtype=np.uint8)
    ne, fa, no = _f32(nears), _f32(fars), _f32(noises)
    n = o.shape[0]
    counts = np.empty(n, np.int32)
    args = (_p(o), _p(d), _p(bf), _f(bound), _f(dt_gamma), _u32(max_steps), _u32(n), _u32(C),
            _u32(H), _p(ne), _p(fa), _p(no), _p(counts))
    total = lib().orc_march_rays_train(*args, None, None, None)
    xyzs = np.zeros((total, 3), np.float32)
    dirs = np.zeros((total, 3), np.float32)
    deltas = np.zeros((total, 2), np.float32)
    lib().orc_march_rays_train(*args, _p(xyzs), _p(dirs), _p(deltas))
    return counts, xyzs, dirs, deltas


def rays_from_counts(counts):
    counts = np.asarray(counts, np.int64)
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
    return np.stack([np.arange(len(counts)), offs, counts], -1).astype(np.int32)


def composite_rays_train_forward(sigmas, rgbs, deltas, rays, T_thresh=1e-4):
    s, c, dl, r = _f32(sigmas), _f32(rgbs), _f32(deltas), _i32(rays)
    m, n = s.shape[0], r.shape[0]
    ws, depth, image = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
    lib().orc_composite_rays_train_forward(_p(s), _p(c), _p(dl), _p(r), _u32(m), _u32(n),
                                           _f(T_thresh), _p(ws), _p(depth), _p(image))
    return ws, depth, image


def composite_rays_train_backward(grad_ws, grad_image, sigmas, rgbs, deltas, rays, weights_sum,
                                  image, T_thresh=1e-4):
    s, c, dl, r = _f32(sigmas), _f32(rgbs), _f32(deltas), _i32(rays)
    gw, gi, ws, im = _f32(grad_ws), _f32(grad_image), _f32(weights_sum), _f32(image)
    m, n = s.shape[0], r.shape[0]
    gs, gc = np.zeros(m, np.float32), np.zeros((m, 3), np.float32)
    lib().orc_composite_rays_train_backward(_p(gw), _p(gi), _p(s), _p(c), _p(dl), _p(r), _p(ws),
                                            _p(im), _u32(m), _u32(n), _f(T_thresh), _p(gs), _p(gc))
    return gs, gc


def march_rays(n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, dt_gamma, max_steps, C,
               H, bitfield, fars, noises):
    ra, rt = _i32(rays_alive), _f32(rays_t)
    o, d = _f32(rays_o).reshape(-1, 3), _f32(rays_d).reshape(-1, 3)
    bf = np.ascontiguousarray(bitfield, dtype=np.uint8)
    fa, no = _f32(fars), _f32(noises)
    rows = n_alive * n_step
    xyzs, dirs, deltas = (np.zeros((rows, 3), np.float32), np.zeros((rows, 3), np.float32),
                          np.zeros((rows, 2), np.float32))
    lib().orc_march_rays(_u32(n_alive), _u32(n_step), _p(ra), _p(rt), _p(o), _p(d), _f(bound),
                         _f(dt_gamma), _u32(max_steps), _u32(C), _u32(H), _p(bf), _p(fa),
                         _p(xyzs), _p(dirs), _p(deltas), _p(no))
    return xyzs, dirs, deltas


def composite_rays(n_alive, n_step, T_thresh, rays_alive, rays_t, sigmas, rgbs, deltas,
                   weights_sum, depth, image):
    """In place on the (float32 / int32, contiguous) numpy arrays given."""
    for a in (rays_t, weights_sum, depth, image):
        assert a.dtype == np.float32 and a.flags.c_contiguous
    assert rays_alive.dtype == np.int32 and rays_alive.flags.c_contiguous
    s, c, dl = _f32(sigmas), _f32(rgbs), _f32(deltas)
    lib().orc_composite_rays(_u32(n_alive), _u32(n_step), _f(T_thresh), _p(rays_alive),
                             _p(rays_t), _p(s), _p(c), _p(dl), _p(weights_sum), _p(depth),
                             _p(image))


# ---------------------------------------------------------------- gridencoder

_ST = {np.dtype(np.float32): 0, np.dtype(np.float16): 1, np.dtype(np.float64): 2}
_ST_BF16 = 3  # uint16 arrays holding bfloat16 bits (numpy has no bfloat16)


def to_bf16_bits(x):
    """f32 -> bfloat16 bits (uint16), round to nearest even (torch.bfloat16)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x7FFFFF) != 0)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return np.where(nan, ((u >> 16) | 0x40).astype(np.uint16), r)


def bf16_bits_to_f32(b):
    return (np.ascontiguousarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


def round_bf16(x):
    """Round f32 values to bfloat16 (result as f32)."""
    return bf16_bits_to_f32(to_bf16_bits(x))


def _st(a, bf16):
    if bf16:
        if a.dtype != np.uint16:
            raise TypeError("bf16 arrays are passed as uint16 bfloat16 bits")
        return _ST_BF16
    return _ST[a.dtype]


def grid_encode_forward(inputs, embeddings, offsets, S, H, gridtype=1, align_corners=False,
                        calc_dy_dx=False, blc=True, bf16=False):
    """inputs [B, D] f32 in [0,1]; embeddings [rows, C] f32/f16/f64 ->
    outputs [B, L*C] (blc) or [L, B, C] in the embeddings' dtype, dy_dx or None.
    bf16=True: embeddings are uint16 bfloat16 bits, f32 accumulation rounded
    to bf16 once (csrc/field_common.h grid_features); outputs are bf16 bits."""
    x = _f32(inputs)
    emb = np.ascontiguousarray(embeddings)
    st = _st(emb, bf16)
    off = _i32(offsets)
    B, D = x.shape
    C = emb.shape[1]
    L = off.shape[0] - 1
    out = np.zeros((B, L * C) if blc else (L, B, C), emb.dtype)
    dy = np.zeros((B, L * D * C), emb.dtype) if calc_dy_dx else None
    lib().orc_grid_encode_forward(_p(x), _p(emb), ctypes.c_int(st), _p(off), _p(out),
                                  _u32(B), _u32(D), _u32(C), _u32(L), _f(S), _u32(H), _p(dy),
                                  _u32(gridtype), ctypes.c_int(int(align_corners)),
                                  ctypes.c_int(int(blc)))
    return out, dy


def grid_encode_backward(grad, inputs, offsets, C, S, H, gridtype=1, align_corners=False, blc=True,
                         bf16=False):
    """Exact (float64, fixed order) embedding gradient [rows, C] (bf16=True:
    grad holds uint16 bfloat16 bits)."""
    g = np.ascontiguousarray(grad)
    st = _st(g, bf16)
    x = _f32(inputs)
    off = _i32(offsets)
    B, D = x.shape
    L = off.shape[0] - 1
    out = np.zeros((int(off[-1]), C), np.float64)
    lib().orc_grid_encode_backward(_p(g), ctypes.c_int(st), _p(x), _p(off), _p(out),
                                   _u32(B), _u32(D), _u32(C), _u32(L), _f(S), _u32(H),
                                   _u32(gridtype), ctypes.c_int(int(align_corners)),
                                   ctypes.c_int(int(blc)))
    return out


def grid_input_backward(grad, dy_dx, D, C, L, blc=True):
    g, j = _f32(grad), _f32(dy_dx)
    B = j.shape[0]
    out = np.empty((B, D), np.float32)
    lib().orc_grid_input_backward(_p(g), _p(j), _p(out), _u32(B), _u32(D), _u32(C), _u32(L),
                                  ctypes.c_int(int(blc)))
    return out


def round_half(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


# ---------------------------------------------------------------- freqencoder

def freq_encode_forward(inputs, degree):
    x = _f32(inputs)
    B, D = x.shape
    C = D + 2 * D * degree
    out = np.empty((B, C), np.float32)
    lib().orc_freq_encode_forward(_p(x), _u32(B), _u32(D), _u32(degree), _u32(C), _p(out))
    return out


def freq_encode_backward(grad, outputs, D, degree):
    g, o = _f32(grad), _f32(outputs)
    B, C = o.shape
    out = np.empty((B, D), np.float32)
    lib().orc_freq_encode_backward(_p(g), _p(o), _u32(B), _u32(D), _u32(degree), _u32(C), _p(out))
    return out


# ---------------------------------------------------------------- shencoder

def _legendre(l):
    p0, p1 = [Fraction(1)], [Fraction(0), Fraction(1)]
    if l == 0:
        return p0
    for n in range(1, l):
        nxt = [Fraction(0)] * (n + 2)
        for k, c in enumerate(p1):
            nxt[k + 1] += Fraction(2 * n + 1, n + 1) * c
        for k, c in enumerate(p0):
            nxt[k] -= Fraction(n, n + 1) * c
        p0, p1 = p1, nxt
    return p1


def _sh_terms(degree):
    """(index, m, z-polynomial coefficients) of every real SH output, following
    shencoder.cu's ordering l*l + l + m and its Condon-Shortley signs."""
    terms = []
    for l in range(degree):
        for m in range(-l, l + 1):
            am = abs(m)
            poly = _legendre(l)
            for _ in range(am):
                poly = [k * c for k, c in enumerate(poly)][1:] or [Fraction(0)]
            k2 = (2 * l + 1) / (4 * math.pi) * math.factorial(l - am) / math.factorial(l + am)
            norm = math.sqrt(k2) * (math.sqrt(2.0) if am else 1.0) * (-1) ** am
            terms.append((l * l + l + m, m, [norm * float(c) for c in poly]))
    return terms


def sh_encode(inputs, degree):
    """float64 outputs [B, degree^2] and dy_dx [B, 3, degree^2] of shencoder.cu."""
    x = np.asarray(inputs, np.float64)
    X, Y, Z = x[:, 0], x[:, 1], x[:, 2]
    w = X + 1j * Y
    out = np.zeros((x.shape[0], degree * degree))
    jac = np.zeros((x.shape[0], 3, degree * degree))
    for idx, m, q in _sh_terms(degree):
        am = abs(m)
        qz = sum(c * Z ** k for k, c in enumerate(q))
        dqz = sum(k * c * Z ** (k - 1) for k, c in enumerate(q) if k > 0) if len(q) > 1 else 0 * Z
        pw = w ** am
        pw1 = w ** (am - 1) if am > 0 else 0 * w
        if m == 0:
            a, ax, ay = 1.0 + 0 * X, 0 * X, 0 * X
        elif m > 0:
            a, ax, ay = pw.real, am * pw1.real, -am * pw1.imag
        else:
            a, ax, ay = pw.imag, am * pw1.imag, am * pw1.real
        out[:, idx] = a * qz
        jac[:, 0, idx] = ax * qz
        jac[:, 1, idx] = ay * qz
        jac[:, 2, idx] = a * dqz
    return out, jac
