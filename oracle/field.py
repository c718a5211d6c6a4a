"""CPU oracle of the grid NeRF field under fp16 autocast — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.

Restates, in numpy, what the reference computes when `common_forward`
(nerf/network_grid.py:76-87) runs under `torch.autocast(fp16)`
(nerf/utils.py:346-399 wraps train_step in autocast with -O):

* grid features: GridEncoder with the f32 embeddings cast to f16 by autocast
  (gridencoder/grid.py:38-39), f16 accumulation per corner
  (gridencoder.cu:142,165) -> the C oracle (`oracle.grid_encode_forward`);
* MLP (network_grid.py:13-32): each nn.Linear under autocast is an f16 GEMM
  (f16 inputs, f16 weight and bias, f32 accumulation, f16 output), ReLU on the
  f16 values.  The oracle forms every dot product EXACTLY (float64: f16
  products are exact in f64 and a 64-term sum of them carries ~30 spare bits),
  rounds it to f32 and then to f16 — the value an f32-accumulating GEMM
  produces whenever its own summation error does not cross an f16 rounding
  boundary.  A GPU result may therefore differ from this oracle by one f16 ulp
  on a small fraction of activations; the tests bound that fraction;
* sigma = trunc_exp(h0 + gaussian(x)) with h0 the f16 output promoted to f32
  (activation.py:5-12 casts to f32), gaussian in f32 (network_grid.py:69-74);
  albedo = sigmoid(h[1:4]) on the f16 tensor (f32 opmath, f16 result);
* backward (autograd of the same graph): trunc_exp' = g exp(clamp(y, -15,
  15)) in f32 (activation.py:14-18), rounded to f16 where it enters the f16
  tensor h0; sigmoid_backward g (1 - y) y in f32 opmath rounded to f16; each
  Linear's input gradient dY W as an f16 GEMM (exact sum -> f32 -> f16), the
  ReLU mask from the f16 outputs; the weight and bias gradients are returned
  as EXACT float64 sums over the samples of the f16 operands (the reference
  rounds them to f16 before autocast's cast back to f32; the product path keeps
  f32 — both lie within one f16 ulp of this value).

The same restatement under bf16 autocast (the C5 option; the reference has
no bf16 path) is selected with `with precision("bf16"):` — every rounding
point above rounds to bfloat16 instead (values kept as f32 arrays holding
bf16 numbers), the grid features accumulate in f32 and round once
(`encode_bf16`), and the windows use bf16's spacing (2^-7 relative).

The background network (network_grid.py:158-167: FreqEncoder -> 39 -> 64 -> 3
MLP -> sigmoid) and the per-ray tail of run_cuda (renderer.py:536-551) are
restated the same way.
"""
from __future__ import annotations

import contextlib

import numpy as np

from . import (bf16_bits_to_f32, freq_encode_forward, grid_encode_forward, round_bf16,
               to_bf16_bits)

F16, F32, F64 = np.float16, np.float32, np.float64

# the autocast element type of the field restatement: "f16" (the reference's
# fp16 autocast) or "bf16" (values stored as f32 arrays of bf16 numbers)
_ELEM = {"name": "f16"}


@contextlib.contextmanager
def precision(name):
    """Select the element type ("f16" or "bf16") of r16 / relu16 / ulp16 and
    the field forward / backward / window functions built on them."""
    if name not in ("f16", "bf16"):
        raise ValueError(name)
    prev, _ELEM["name"] = _ELEM["name"], name
    try:
        yield
    finally:
        _ELEM["name"] = prev


def _vd():
    return F16 if _ELEM["name"] == "f16" else F32


def r16(x):
    """Round to the element type (f16, or bf16 under precision("bf16")),
    round-to-nearest-even, via f32 like an f32 accumulator."""
    if _ELEM["name"] == "bf16":
        return round_bf16(np.asarray(x).astype(F32))
    return np.asarray(x).astype(F32).astype(F16)


def linear16(x16, w, b, chunk=None):
    """nn.Linear under fp16 autocast: f16 x [M, K] @ f16(w)[N, K]^T + f16(b).

    chunk=None: the exactly-rounded dot product (reference semantics, any
    f32-accumulating GEMM up to its own rounding).  chunk=k: the accumulation
    model of an MFMA chain — the f32 accumulator starts at the bias and each
    instruction adds the exact sum of its k products with ONE f32 rounding
    (csrc/fieldmlp.hip forward_tile: k = 32, K = 32 or 64)."""
    x = x16.astype(F64)
    w16 = r16(w).astype(F64)
    b16 = r16(b).astype(F64) if b is not None else 0.0
    if chunk is None:
        return r16(x @ w16.T + b16)
    acc = np.broadcast_to(np.asarray(b16, F64), (x.shape[0], w16.shape[0])).astype(F32)
    for k0 in range(0, x.shape[1], chunk):
        acc = (acc.astype(F64) + x[:, k0:k0 + chunk] @ w16[:, k0:k0 + chunk].T).astype(F32)
    return r16(acc)


def relu16(z16):
    return np.where(z16 > 0, z16, 0).astype(_vd())


def gaussian(x):
    """network_grid.py:69-74 in f32: 5 * exp(-(x**2).sum(-1) / (2 * 0.2**2))."""
    x = np.asarray(x, F32)
    s = (x[:, 0] * x[:, 0] + x[:, 1] * x[:, 1]) + x[:, 2] * x[:, 2]
    return (F32(5.0) * np.exp(-(s / F32(0.08)).astype(F64)).astype(F32)).astype(F32)


def sigmoid16(h16):
    h = h16.astype(F64)
    return r16(1.0 / (1.0 + np.exp(-h)))


def encode(xyz, bound, embeddings, offsets, S, H):
    """f16 grid features [M, 32] of positions xyz in [-bound, bound]
    (grid.py:142 maps them to [0, 1] in f32)."""
    x01 = ((np.asarray(xyz, F32) + F32(bound)) / F32(2 * bound)).astype(F32)
    out, _ = grid_encode_forward(x01, np.asarray(embeddings).astype(F16), offsets, S, H)
    return out


def encode_bf16(xyz, bound, embeddings, offsets, S, H):
    """bf16 grid features [M, 32] (as f32 values): the f32 embeddings rounded to
    bf16, f32 accumulation per corner (fmaf, corner order), one rounding."""
    x01 = ((np.asarray(xyz, F32) + F32(bound)) / F32(2 * bound)).astype(F32)
    out, _ = grid_encode_forward(x01, to_bf16_bits(np.asarray(embeddings, F32)), offsets, S, H,
                                 bf16=True)
    return bf16_bits_to_f32(out)


def field_forward(xyz, weights, enc16, chunk=None):
    """common_forward from the features: weights = (w1, b1, w2, b2, w3, b3)
    f32 arrays (nn.Linear layout); chunk: see linear16.  Returns a dict with
    the f16 activations, h [M, 4] f16, y = f32(h0) + gaussian, sigma f32 and
    albedo f16."""
    w1, b1, w2, b2, w3, b3 = weights
    a1 = relu16(linear16(enc16, w1, b1, chunk))
    a2 = relu16(linear16(a1, w2, b2, chunk))
    h = linear16(a2, w3, b3, chunk)
    y = (h[:, 0].astype(F32) + gaussian(xyz)).astype(F32)
    sigma = np.exp(y.astype(F64)).astype(F32)
    albedo = sigmoid16(h[:, 1:])
    return {"x": enc16, "a1": a1, "a2": a2, "h": h, "y": y, "sigma": sigma, "albedo": albedo}


def field_backward(fwd, weights, grad_sigma, grad_albedo16):
    """Backward of field_forward for upstream gradients grad_sigma [M] f32
    and grad_albedo16 [M, 3] f16.  Returns a dict: d_enc [M, 32] f16, grads =
    [dW1, db1, dW2, db2, dW3, db3] float64 exact sums, and the f16 gradients
    dO [M, 4], dz2, dz1 and their pre-mask f64 sums dA2, dA1, dX."""
    w1, b1, w2, b2, w3, b3 = (r16(w).astype(F64) for w in weights)
    y = fwd["y"]
    yc = np.clip(y, F32(-15), F32(15))
    d0 = r16(np.asarray(grad_sigma, F32) * np.exp(yc.astype(F64)).astype(F32))
    a = fwd["albedo"].astype(F32)
    g = np.asarray(grad_albedo16).astype(_vd()).astype(F32)
    drgb = r16((g * (F32(1) - a)) * a)
    dO = np.concatenate([d0[:, None], drgb], axis=1).astype(_vd())
    dA2 = dO.astype(F64) @ w3
    dz2 = np.where(fwd["a2"] > 0, r16(dA2), 0).astype(_vd())
    dA1 = dz2.astype(F64) @ w2
    dz1 = np.where(fwd["a1"] > 0, r16(dA1), 0).astype(_vd())
    dX = dz1.astype(F64) @ w1
    x64, a1, a2 = fwd["x"].astype(F64), fwd["a1"].astype(F64), fwd["a2"].astype(F64)
    dO64, dz2_64, dz1_64 = dO.astype(F64), dz2.astype(F64), dz1.astype(F64)
    grads = [dz1_64.T @ x64, dz1_64.sum(0), dz2_64.T @ a1, dz2_64.sum(0), dO64.T @ a2,
             dO64.sum(0)]
    return {"d_enc": r16(dX), "grads": grads, "dO": dO, "dz2": dz2, "dz1": dz1, "dA2": dA2,
            "dA1": dA1, "dX": dX, "grad_sigma": np.asarray(grad_sigma, F32), "g16": g}


# ------------------------------------------------- error bounds of any correct GPU result
#
# An f16-autocast GEMM accumulating in f32 (any order, MFMA or not) returns,
# for each output, r16 of a value within gamma_K * sum|terms| of the exact dot
# product (gamma_K = (K + 2) u, u = 2^-24: the standard bound for K
# products + the bias).  Where that window contains an f16 rounding boundary
# the result may be the neighbouring f16 value, and the difference propagates
# into the later layers.  The functions below propagate these windows through
# the forward and the backward of the field: every GPU output must lie inside
# them.  Outside the windows the GPU value must equal the oracle's bit for
# bit, so for most samples the bound is exactly zero.

U32 = 2.0 ** -24


# f32 accumulation model of the GEMMs: None = the rigorous bound for ANY
# summation order, (K + 2) u; an int c = c u, the model of an MFMA chain
# (each v_mfma_f32_16x16x32_f16 sums its 32 products internally and rounds
# into the f32 accumulator once: 2-3 roundings for K <= 64; 8 leaves margin).
ACC_ULPS = None


def _gamma(k, acc_ulps=None):
    return (k + 2 if acc_ulps is None else acc_ulps) * U32


def _round_window(z, dz, post=None):
    """Largest |post(r16(z')) - post(r16(z))| over |z' - z| <= dz (r16 and the
    optional monotone post-op are monotone, so the window's ends suffice)."""
    post = post or (lambda v: v)
    mid = post(r16(z).astype(F64))
    lo = post(r16(z - dz).astype(F64))
    hi = post(r16(z + dz).astype(F64))
    return np.maximum(np.abs(hi - mid), np.abs(mid - lo))


def _relu(v):
    return np.maximum(v, 0.0)


def _layer_window(x, dx, w, b, z, acc_ulps=None):
    """Error window of z = x @ w16^T + b16 computed in f32 from inputs that may
    be off by dx: |w| dx + gamma_K (|x| + dx) |w| + gamma |b|."""
    aw = np.abs(r16(w).astype(F64))
    ab = np.abs(r16(b).astype(F64)) if b is not None else 0.0
    k = aw.shape[1]
    return dx @ aw.T + _gamma(k, acc_ulps) * ((np.abs(x) + dx) @ aw.T + ab)


def forward_bounds(fwd, weights, acc_ulps=None):
    """Per-sample windows of the forward: da1 [M, 64], da2 [M, 64], dh [M, 4]
    (f16 outputs of the layers), dlog_sigma [M], dalbedo [M, 3].  acc_ulps:
    the GEMMs' f32 accumulation model (see _gamma)."""
    w1, b1, w2, b2, w3, b3 = weights
    x = fwd["x"].astype(F64)
    z1 = x @ r16(w1).astype(F64).T + r16(b1).astype(F64)
    da1 = _round_window(z1, _layer_window(x, np.zeros_like(x), w1, b1, z1, acc_ulps), _relu)
    a1 = fwd["a1"].astype(F64)
    z2 = a1 @ r16(w2).astype(F64).T + r16(b2).astype(F64)
    da2 = _round_window(z2, _layer_window(a1, da1, w2, b2, z2, acc_ulps), _relu)
    a2 = fwd["a2"].astype(F64)
    z3 = a2 @ r16(w3).astype(F64).T + r16(b3).astype(F64)
    dz3 = _layer_window(a2, da2, w3, b3, z3, acc_ulps)
    dh = _round_window(z3, dz3)
    # sigma = exp(f32(h0) + gaussian): expf / the f32 add / the gaussian add a
    # few f32 ulps of y (|y| <= 16 -> 2^-19 absolute) on top of the h0 window
    y = fwd["y"].astype(F64)
    dlog = dh[:, 0] + 8.0 * U32 * np.maximum(np.abs(y), 1.0)
    # albedo = r16(sigmoid(h)): the window of h, plus one f16 ulp where the
    # f32 sigmoid sits within a few f32 ulps of an f16 rounding boundary
    dalb = _sigmoid16_window(fwd["h"][:, 1:].astype(F64), dh[:, 1:], fwd["albedo"])
    return {"da1": da1, "da2": da2, "dh": dh, "dlog_sigma": dlog, "dalbedo": dalb}


def _sigmoid16_window(h, dh, out16):
    """Window of r16(sigmoid(h')) for f16 h' within dh of h, plus one f16 ulp
    where the f32 sigmoid sits within a few f32 ulps of an f16 rounding
    boundary (expf and the f32 divide are not correctly rounded)."""
    sig = lambda v: 1.0 / (1.0 + np.exp(-v))  # noqa: E731
    lo = r16(sig(r16(h - dh).astype(F64))).astype(F64)
    hi = r16(sig(r16(h + dh).astype(F64))).astype(F64)
    s = sig(h)
    near = r16(s * (1 - 8 * U32)) != r16(s * (1 + 8 * U32))
    o = out16.astype(F64)
    return np.maximum(np.abs(hi - o), np.abs(o - lo)) + np.where(near, ulp16(o), 0.0)


def bg_bounds(fwd, weights, grad_bg=None, sum_gamma=2e-5, acc_ulps=None):
    """Windows of the background network: dbg [N, 3] on the f16 colour, and
    with grad_bg the four weight/bias gradient windows.  The frequency
    features enter with a two-f32-ulp window (sinf vs the oracle's sin)."""
    w1, b1, w2, b2 = weights
    v = freq_encode_forward(np.asarray(fwd["d"], F32), 6).astype(F64)
    dx = _round_window(v, 2 * np.abs(v) * U32 * 2)
    x = fwd["x"].astype(F64)
    z1 = x @ r16(w1).astype(F64).T + r16(b1).astype(F64)
    da1 = _round_window(z1, _layer_window(x, dx, w1, b1, z1, acc_ulps), _relu)
    a1 = fwd["a1"].astype(F64)
    z2 = a1 @ r16(w2).astype(F64).T + r16(b2).astype(F64)
    do_ = _round_window(z2, _layer_window(a1, da1, w2, b2, z2, acc_ulps))
    dbg = _sigmoid16_window(fwd["o"].astype(F64), do_, fwd["bg"])
    out = {"dx": dx, "da1": da1, "do": do_, "dbg": dbg}
    if grad_bg is None:
        return out
    g = np.abs(r16(grad_bg).astype(F64))
    y = fwd["bg"].astype(F64)
    v = r16(grad_bg).astype(F64) * (1 - y) * y
    ddo = _round_window(v, g * (np.abs(1 - 2 * y) * dbg + dbg * dbg) + 4 * U32 * np.abs(v))
    do16 = r16(v).astype(F64)
    aw2 = np.abs(r16(w2).astype(F64))
    dA1 = do16 @ r16(w2).astype(F64)
    ddA1 = ddo @ aw2 + _gamma(64, acc_ulps) * ((np.abs(do16) + ddo) @ aw2)
    ddz1 = _masked_window(a1, da1, dA1, ddA1)
    dz1 = np.abs(np.where(a1 > 0, r16(dA1), 0).astype(F64))
    ax, aa1, ado = np.abs(x), np.abs(a1), np.abs(do16)

    def wwin(ad, dd, act, dact):
        return (dd.T @ act + ad.T @ dact + dd.T @ dact) + sum_gamma * ((ad + dd).T @ (act + dact))

    out["grads"] = [wwin(dz1, ddz1, ax, dx), ddz1.sum(0) + sum_gamma * (dz1 + ddz1).sum(0),
                    wwin(ado, ddo, aa1, da1), ddo.sum(0) + sum_gamma * (ado + ddo).sum(0)]
    return out


def mlp_forward(x16, weights, acc_ulps=None, dx=None):
    """Generic nn.Linear/ReLU stack under fp16 autocast (network_grid.py:13-32:
    ReLU between layers, none after the last).  weights = [w0, b0, w1, b1,
    ...].  Returns (outputs, windows): the f16 output of every layer and the
    propagated window of each (dx: window of the inputs, default exact)."""
    a = np.asarray(x16, F16)
    da = np.zeros(a.shape) if dx is None else dx
    outs, wins = [], []
    n = len(weights) // 2
    for i in range(n):
        w, b = weights[2 * i], weights[2 * i + 1]
        a64 = a.astype(F64)
        z = a64 @ r16(w).astype(F64).T + (r16(b).astype(F64) if b is not None else 0.0)
        dz = _layer_window(a64, da, w, b, z, acc_ulps)
        last = i == n - 1
        a = r16(z) if last else relu16(r16(z))
        da = _round_window(z, dz, None if last else _relu)
        outs.append(a)
        wins.append(da)
    return outs, wins


def ulp16(v):
    """Spacing of f16 values at |v| (subnormal spacing 2^-24 below 2^-14); of
    bf16 values (2^-7 relative) under precision("bf16")."""
    a = np.abs(np.asarray(v, F64))
    if _ELEM["name"] == "bf16":
        return np.exp2(np.floor(np.log2(np.maximum(a, 2.0 ** -126)))) * 2.0 ** -7
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -14)))
    return np.exp2(e) * 2.0 ** -10


def _masked_window(act, dact, pre, dpre):
    """Window of dz = (act > 0) ? r16(pre) : 0 when act may be off by dact and
    pre by dpre: a mask that can flip costs the whole |r16(pre)| + dpre."""
    win = _round_window(pre, dpre)
    # act >= 0 (post-ReLU); the GPU's value lies in [act - dact, act + dact]
    can_flip = np.where(act > 0, act - dact <= 0, dact > 0)
    val = np.abs(r16(pre).astype(F64)) + dpre + win
    return np.where(can_flip, val, np.where(act > 0, win, 0.0))


def backward_bounds(fwd, fb, weights, fwd_bounds, sum_gamma=2e-5, acc_ulps=None):
    """Windows of the backward: d_enc [M, 32] (f16 feature gradients) and the
    six weight/bias gradients (absolute, elementwise).  sum_gamma bounds the
    relative error of an f32 reduction over the samples in any blocked order."""
    w1, b1, w2, b2, w3, b3 = weights
    fb_ = fwd_bounds
    # dO0 = r16(gs * exp(clamp(y))): y off by dlog_sigma; expf and the product
    # add 3 f32 ulps
    gs = np.abs(fb["grad_sigma"].astype(F64))
    yc = np.clip(fwd["y"].astype(F64), -15, 15)
    e = np.exp(yc)
    v0 = fb["grad_sigma"].astype(F64) * e
    d0 = gs * e * (np.expm1(fb_["dlog_sigma"]) + 4 * U32)
    dd0 = _round_window(v0, d0)
    # dO_rgb = r16(g (1 - a) a): a off by dalbedo
    g = fb["g16"].astype(F64)
    a = fwd["albedo"].astype(F64)
    da = fb_["dalbedo"]
    vr = g * (1 - a) * a
    dr = np.abs(g) * (np.abs(1 - 2 * a) * da + da * da) + 4 * U32 * np.abs(vr)
    ddr = _round_window(vr, dr)
    ddO = np.concatenate([dd0[:, None], ddr], axis=1)
    dO = fb["dO"].astype(F64)
    aw3, aw2, aw1 = (np.abs(r16(w).astype(F64)) for w in (w3, w2, w1))
    # layer 3 backward: dA2 = dO W3 (K = 4 nonzero terms)
    ddA2 = ddO @ aw3 + _gamma(4, acc_ulps) * ((np.abs(dO) + ddO) @ aw3)
    ddz2 = _masked_window(fwd["a2"].astype(F64), fb_["da2"], fb["dA2"], ddA2)
    dz2 = fb["dz2"].astype(F64)
    ddA1 = ddz2 @ aw2 + _gamma(64, acc_ulps) * ((np.abs(dz2) + ddz2) @ aw2)
    ddz1 = _masked_window(fwd["a1"].astype(F64), fb_["da1"], fb["dA1"], ddA1)
    dz1 = fb["dz1"].astype(F64)
    ddX = ddz1 @ aw1 + _gamma(64, acc_ulps) * ((np.abs(dz1) + ddz1) @ aw1)
    dd_enc = _round_window(fb["dX"], ddX)
    # weight gradients: sum_m dz[m] act[m] with both factors windowed
    x = np.abs(fwd["x"].astype(F64))
    a1, a2 = np.abs(fwd["a1"].astype(F64)), np.abs(fwd["a2"].astype(F64))
    da1, da2 = fb_["da1"], fb_["da2"]
    adz1, adz2, adO = np.abs(dz1), np.abs(dz2), np.abs(dO)

    def wwin(ad, dd, act, dact):
        return (dd.T @ act + ad.T @ dact + dd.T @ dact) + sum_gamma * ((ad + dd).T @ (act + dact))

    def bwin(ad, dd):
        return dd.sum(0) + sum_gamma * (ad + dd).sum(0)

    z = np.zeros_like(x)
    grads = [wwin(adz1, ddz1, x, z), bwin(adz1, ddz1), wwin(adz2, ddz2, a1, da1),
             bwin(adz2, ddz2), wwin(adO, ddO, a2, da2), bwin(adO, ddO)]
    return {"d_enc": dd_enc, "grads": grads, "dO": ddO}


# ----------------------------------------------------------------- background + ray tail

def bg_forward(rays_d, weights):
    """background(d) (network_grid.py:158-167) under autocast: freq encoding in
    f32 (freqencoder.cu:28-58, degree 6), cast to f16, 39 -> 64 -> 3 f16
    Linear layers with ReLU, sigmoid -> f16 colour [N, 3]."""
    w1, b1, w2, b2 = weights
    x = r16(freq_encode_forward(np.asarray(rays_d, F32), 6))
    a1 = relu16(linear16(x, w1, b1))
    o = linear16(a1, w2, b2)
    return {"d": np.asarray(rays_d, F32), "x": x, "a1": a1, "o": o, "bg": sigmoid16(o)}


def bg_backward(fwd, weights, grad_bg):
    """grad_bg [N, 3] f32 (the f32 mix's gradient) -> exact float64 [dW1,
    db1, dW2, db2] of the f16 graph."""
    w1, b1, w2, b2 = (r16(w).astype(F64) for w in weights)
    g = r16(grad_bg).astype(F32)  # autocast: gradient of the f16 sigmoid output
    y = fwd["bg"].astype(F32)
    do = r16((g * (F32(1) - y)) * y)
    dz1 = np.where(fwd["a1"] > 0, r16(do.astype(F64) @ w2), F16(0)).astype(F16)
    do64, dz1_64 = do.astype(F64), dz1.astype(F64)
    return [dz1_64.T @ fwd["x"].astype(F64), dz1_64.sum(0), do64.T @ fwd["a1"].astype(F64),
            do64.sum(0)]


def ray_tail(ws, depth, image, nears, fars, bg):
    """renderer.py:536-551: image + (1 - ws) bg, clamp(depth - near, 0) /
    (far - near), mask near < far — all f32."""
    ws, depth, nears, fars = (np.asarray(a, F32) for a in (ws, depth, nears, fars))
    img = (np.asarray(image, F32) + (F32(1) - ws)[:, None] * np.asarray(bg, F32)).astype(F32)
    d = (np.maximum(depth - nears, F32(0)) / (fars - nears)).astype(F32)
    return img, d, nears < fars


def entropy(ws, lam):
    """utils.py:386-391: lam * mean(-a log2 a - (1-a) log2(1-a)), a = clamp(ws,
    1e-5, 1-1e-5); returns (loss f64, d loss / d ws f64)."""
    w = np.asarray(ws, F64)
    a = np.clip(w, 1e-5, 1 - 1e-5)
    e = -a * np.log2(a) - (1 - a) * np.log2(1 - a)
    inside = (w >= 1e-5) & (w <= 1 - 1e-5)
    g = np.where(inside, lam / w.size * (np.log2(1 - a) - np.log2(a)), 0.0)
    return lam * e.mean(), g


# ----------------------------------------------------------------- shading (non-albedo steps)

def fd_normal(sig_pm, eps=1e-2):
    """network_grid.py:90-121 in f32: sig_pm [6, M] = sigma at x + eps e_a
    (rows +x, -x, +y, -y, +z, -z) -> (v [M, 3], normal [M, 3], |v|^2, r, nan
    mask): v = -(0.5 (s+ - s-) / eps), normal = v / sqrt(clamp(|v|^2, 1e-20)),
    NaN -> 0."""
    s = np.asarray(sig_pm, F32)
    e = F32(eps)
    v = np.stack([-((F32(0.5) * (s[2 * a] - s[2 * a + 1])) / e) for a in range(3)], -1)
    v = v.astype(F32)
    ss = ((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]).astype(F32)
    r = np.sqrt(np.maximum(ss, F32(1e-20))).astype(F32)
    with np.errstate(invalid="ignore", divide="ignore"):
        n = (v / r[:, None]).astype(F32)
    nan = np.isnan(n)
    return v, np.where(nan, F32(0), n).astype(F32), ss, r, nan


def shade_forward(sigma, sig_pm, albedo16, dirs, light, ratio, shading, eps=1e-2):
    """network_grid.py:124-144 + renderer.py:485-489 under autocast: returns a
    dict with normal [M, 3] f32, dot16 / lam16 [M] f16, color [M, 3] f16 and
    the per-sample orientation terms [M] f32 (w.detach() * clamp(n.d, 0)^2)."""
    v, n, ss, r, nan = fd_normal(sig_pm, eps)
    l16 = r16(light).astype(F64)
    # normal @ l: f16 operands (products exact), f32 sum, f16 result
    p = r16(n).astype(F64) * l16[None, :]
    d16 = r16(((p[:, 0] + p[:, 1]) + p[:, 2]).astype(F32))
    c16 = np.maximum(d16.astype(F32), F32(0))
    omr = F32(1.0 - float(ratio))
    lam16 = r16(F32(ratio) + r16(c16 * omr).astype(F32))
    if shading == "textureless":
        color = np.repeat(lam16[:, None], 3, 1)
    else:  # lambertian
        color = r16(np.asarray(albedo16).astype(_vd()).astype(F32) * lam16.astype(F32)[:, None])
    w = (F32(1) - np.exp(-np.asarray(sigma, F32).astype(F64)).astype(F32)).astype(F32)
    d = np.asarray(dirs, F32)
    nd = ((n[:, 0] * d[:, 0] + n[:, 1] * d[:, 1]) + n[:, 2] * d[:, 2]).astype(F32)
    c = np.maximum(nd, F32(0))
    orient = (w * (c * c)).astype(F32)
    return {"v": v, "normal": n, "ss": ss, "r": r, "nan": nan, "d16": d16, "lam16": lam16,
            "color": color.astype(_vd()), "w": w, "nd": nd, "orient": orient, "l16": l16}


def padded_rows(m):
    """The march's returned row count M' (raymarching.py:224-227)."""
    return m + 128 - m % 128


def shade_backward(fwd, albedo16, dirs, grad_color16, grad_loss, lam_orient, m_rows, ratio,
                   shading, eps=1e-2):
    """Autograd of shade_forward for the f16 colour gradient grad_color16
    [M, 3] and the loss-scale upstream grad_loss of lam_orient * mean(orient)
    over m_rows (= M').  Returns (grad_sig_pm [6, M] f32, grad_albedo16 [M, 3]
    f16 or None)."""
    g = np.asarray(grad_color16).astype(_vd()).astype(F32)
    lam = fwd["lam16"].astype(F32)
    ga = None
    if shading == "textureless":
        glam = r16((g[:, 0] + g[:, 1]) + g[:, 2]).astype(F32)
    else:
        a = np.asarray(albedo16).astype(_vd()).astype(F32)
        ga = r16(g * lam[:, None])
        gl = r16(g * a).astype(F32)
        glam = r16((gl[:, 0] + gl[:, 1]) + gl[:, 2]).astype(F32)
    gc = r16(glam * F32(1.0 - float(ratio))).astype(F32)
    gd = np.where(fwd["d16"] >= 0, gc, F32(0)).astype(F32)
    gn = r16(gd[:, None] * fwd["l16"].astype(F32)[None, :]).astype(F32)
    go = F32((F32(grad_loss) * F32(lam_orient)) / F32(m_rows))
    d = np.asarray(dirs, F32)
    g2 = np.where(fwd["nd"] >= 0, (go * fwd["w"]) * (F32(2) * np.maximum(fwd["nd"], F32(0))),
                  F32(0)).astype(F32)
    gn = (gn + g2[:, None] * d).astype(F32)
    gn = np.where(fwd["nan"], F32(0), gn)
    v, r, ss = fwd["v"], fwd["r"], fwd["ss"]
    r2 = (r * r).astype(F32)
    gr = ((((-gn[:, 0] * v[:, 0]) / r2) + ((-gn[:, 1] * v[:, 1]) / r2)) +
          ((-gn[:, 2] * v[:, 2]) / r2)).astype(F32)
    gs = np.where(ss >= F32(1e-20), gr / (F32(2) * r), F32(0)).astype(F32)
    gv = (gn / r[:, None] + (gs[:, None] * v + gs[:, None] * v)).astype(F32)
    gdiff = (F32(0.5) * (-gv / F32(eps))).astype(F32)
    out = np.empty((6, gv.shape[0]), F32)
    for a in range(3):
        out[2 * a] = gdiff[:, a]
        out[2 * a + 1] = -gdiff[:, a]
    return out, ga


# ----------------------------------------------------------------- backward structures of the step
#
# The reference runs TWO backward passes per train step: nerf/sd.py:115
# `latents.backward(gradient=grad, retain_graph=True)` carries the UNSCALED SDS
# gradient down the render graph, then nerf/utils.py:708
# `scaler.scale(loss).backward()` carries the loss-scaled regulariser
# gradient; autograd's AccumulateGrad adds the second pass's parameter
# gradients onto the first's in f32.  The fused structure (this package's
# headline, Trainer.fused_backward) runs ONE backward with both upstream
# gradients summed where they meet — at weights_sum, in f32 — so every f16
# rounding point of the field backward (dO = r16(...), dz2, dz1, d_enc) rounds
# the SUM once instead of each pass's part separately.  Both are restated
# here on top of the compositing backward (oracle.c) and field_backward.

def step_upstreams(structure, grad_ws_sds, grad_ws_loss, grad_image):
    """Upstream gradients at the compositing outputs, one (grad_ws [N],
    grad_image [N, 3]) pair per backward pass: "fused" -> one pass with the
    weights-sum gradients added in f32; "two_pass" -> the SDS pass (image and
    its weights-sum gradient) then the loss pass (weights-sum only)."""
    gs, gl = np.asarray(grad_ws_sds, F32), np.asarray(grad_ws_loss, F32)
    gi = np.asarray(grad_image, F32)
    if structure == "fused":
        return [((gs + gl).astype(F32), gi)]
    if structure == "two_pass":
        return [(gs, gi), (gl, np.zeros_like(gi))]
    raise ValueError(structure)


def composite_backward(grad_ws, grad_image, sigma, rgb16, deltas, rays, ws, image):
    """One pass of the compositing backward (raymarching.cu:601-693 via
    oracle.c, f32): (grad_sigma f32 [M], grad_albedo [M, 3] rounded to the
    element type, as autocast's cast backward delivers it to the f16 / bf16
    albedo)."""
    from . import composite_rays_train_backward
    gs, gc = composite_rays_train_backward(grad_ws, grad_image, sigma,
                                           np.asarray(rgb16).astype(F32), deltas, rays, ws,
                                           image)
    return gs, r16(gc)


def backward_passes(fwd, weights, passes):
    """field_backward of every pass [(grad_sigma, grad_albedo16), ...]:
    returns {"passes": [bo, ...], "d_enc": [d_enc of each pass], "grads": the
    six parameter gradients summed over the passes (each pass exact in f64;
    AccumulateGrad's f32 add is within the windows of backward_pass_bounds)}."""
    bos = [field_backward(fwd, weights, gs, ga) for gs, ga in passes]
    grads = [sum(bo["grads"][i] for bo in bos) for i in range(6)]
    return {"passes": bos, "d_enc": [bo["d_enc"] for bo in bos], "grads": grads}


def backward_pass_bounds(fwd, bp, weights, fwd_bounds, acc_ulps=None):
    """Windows of backward_passes: per-pass d_enc windows, and the summed
    parameter gradients' windows (the passes' windows added, plus one f32
    rounding of the running sum per pass)."""
    bbs = [backward_bounds(fwd, bo, weights, fwd_bounds, acc_ulps=acc_ulps)
           for bo in bp["passes"]]
    grads = []
    for i in range(6):
        w = sum(bb["grads"][i] for bb in bbs)
        mag = sum(np.abs(bo["grads"][i]) for bo in bp["passes"])
        grads.append(w + len(bbs) * U32 * (mag + w))
    return {"passes": bbs, "d_enc": [bb["d_enc"] for bb in bbs], "grads": grads}


def f16_underflow(fwd, bo):
    """How much of a pass's f16 backward falls out of the element type's
    normal range: for the first rounding point dO = r16(grad_sigma exp(y)),
    r16(g (1 - a) a) and for the feature gradients d_enc = r16(dX), the
    fraction of entries whose exact value is nonzero but below 2^-14 (f16
    subnormal: fewer than 11 significant bits) and the fraction that round to
    zero.  Returns a dict of those four fractions."""
    yc = np.clip(fwd["y"].astype(F64), -15, 15)
    e0 = bo["grad_sigma"].astype(F64) * np.exp(yc)
    a = fwd["albedo"].astype(F64)
    er = bo["g16"].astype(F64) * (1 - a) * a
    exact_o = np.concatenate([e0[:, None], er], 1)
    out = {}
    for name, exact, rounded in (("dO", exact_o, bo["dO"]), ("d_enc", bo["dX"], bo["d_enc"])):
        ex = np.abs(exact)
        nz = ex > 0
        n = max(int(nz.sum()), 1)
        out[name + "_subnormal"] = float(((ex < 2.0 ** -14) & nz).sum() / n)
        out[name + "_zero"] = float(((rounded == 0) & nz).sum() / n)
    return out
