"""Shared oracle comparisons for the GPU field tests (imported by test
modules; not collected itself).  See tests/test_gpu_field_oracle.py for the
tolerance model: every GPU value must lie inside the oracle's propagated
f16-rounding window (oracle/field.py), which is closed — i.e. bit-exact — for
most values."""
import numpy as np

import oracle
import oracle.field as of

# forward GEMMs: MFMA chains, few f32 roundings (oracle.field._gamma)
MFMA_ULPS = 8


def embedding_window(d_enc, d_enc_win, x01, offsets, S, H):
    """|grad_embeddings| window: the corner weights are non-negative, so the
    backward of the feature-gradient window bounds the propagated error; the
    f64-accumulated, once-rounded product path adds one f32 rounding plus the
    f16 products' own rounding (2^-22 of the |term| sum)."""
    M = d_enc.shape[0]
    win = oracle.grid_encode_backward(np.asarray(d_enc_win, np.float32).reshape(M, 16, 2), x01,
                                      offsets, 2, S, H)
    mag = oracle.grid_encode_backward(np.abs(d_enc.astype(np.float32)).reshape(M, 16, 2), x01,
                                      offsets, 2, S, H)
    return np.abs(win) + 2.0 ** -22 * mag


def check_field(xyz, emb, offsets, S, H, weights, sigma, albedo, grad_sigma=None,
                grad_albedo16=None, grads=None, grad_emb=None, label="", bf16=False):
    """Compare one GPU field evaluation (and optionally its backward) with the
    oracle.  Arrays are numpy; weights = the six f32 MLP tensors; grads = the
    six GPU gradients; grad_emb = the GPU embedding gradient.  bf16: the bf16
    autocast restatement (oracle.field.precision("bf16"); albedo and
    grad_albedo16 then hold bf16 values as f32).  Returns a dict of
    statistics (printed by the callers)."""
    with of.precision("bf16" if bf16 else "f16"):
        return _check_field(xyz, emb, offsets, S, H, weights, sigma, albedo, grad_sigma,
                            grad_albedo16, grads, grad_emb, label, bf16)


def _check_field(xyz, emb, offsets, S, H, weights, sigma, albedo, grad_sigma, grad_albedo16,
                 grads, grad_emb, label, bf16):
    M = xyz.shape[0]
    stats = {"M": M}
    x16 = (of.encode_bf16 if bf16 else of.encode)(xyz, 1.0, emb, offsets, S, H)
    fo = of.field_forward(xyz, weights, x16)
    fb = of.forward_bounds(fo, weights, acc_ulps=MFMA_ULPS)
    dlog = np.abs(np.log(sigma.astype(np.float64)) - np.log(fo["sigma"].astype(np.float64)))
    assert np.all(dlog <= fb["dlog_sigma"]), \
        f"{label} sigma outside its window by {(dlog - fb['dlog_sigma']).max():.3e}"
    da = np.abs(albedo.astype(np.float64) - fo["albedo"].astype(np.float64))
    assert np.all(da <= fb["dalbedo"]), \
        f"{label} albedo outside its window by {(da - fb['dalbedo']).max():.3e}"
    stats["h0_differs"] = float(np.mean(
        dlog > 8 * 2.0 ** -24 * np.maximum(np.abs(fo["y"].astype(np.float64)), 1.0)))
    stats["albedo_differs"] = float(np.mean((da > 0).any(1))) if M else 0.0
    if grads is None:
        return stats
    bo = of.field_backward(fo, weights, grad_sigma, grad_albedo16)
    bb = of.backward_bounds(fo, bo, weights, fb, acc_ulps=None)
    d_win = bb["d_enc"]
    if not bf16:  # f16 subnormal allowance, see test_gpu_field_oracle.py
        sub = np.abs(bo["d_enc"].astype(np.float64)) < 2.0 ** -14
        d_win = d_win + np.where(sub, 2.0 ** -24, 0.0)
    for i, (a, b, w) in enumerate(zip(grads, bo["grads"], bb["grads"])):
        a = np.asarray(a, np.float64).reshape(b.shape)
        err = np.abs(a - b)
        assert np.all(err <= w), f"{label} MLP param {i} outside its window by {(err - w).max():.3e}"
    if grad_emb is not None:
        x01 = ((np.asarray(xyz, np.float32) + np.float32(1)) / np.float32(2)).astype(np.float32)
        want = oracle.grid_encode_backward(bo["d_enc"].astype(np.float32).reshape(M, 16, 2), x01,
                                           offsets, 2, S, H)
        win = embedding_window(bo["d_enc"], d_win, x01, offsets, S, H)
        err = np.abs(np.asarray(grad_emb, np.float64) - want)
        assert np.all(err <= win + 1e-30), \
            f"{label} embedding grads outside their window by {(err - win).max():.3e}"
        stats["emb_rel_norm"] = float(np.linalg.norm(err) / max(np.linalg.norm(want), 1e-30))
    return stats
