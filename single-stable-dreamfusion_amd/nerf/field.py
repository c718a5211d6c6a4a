"""Fused grid field: tiled-grid encoding + sigma MLP + density/albedo heads as
ONE autograd node on the native kernels (the reference's
network_grid.common_forward, nerf/network_grid.py:76-87, = GridEncoder ->
MLP -> trunc_exp(h0 + gaussian) / sigmoid(h[1:])).

Forward: grid_encode_forward_blc (f16 features) -> field_mlp_forward (MFMA).
Backward: field_mlp_backward (recomputes the MLP from the saved features,
writes the feature gradient straight into the [L, B, C] layout) ->
grid_encode_backward_sliced.  Used under fp16 autocast for the reference's
network shape (16 levels x 2 channels, 32 -> 64 -> 64 -> 4); anything else
runs the unfused modules.
"""
import numpy as np
import torch
from torch.autograd import Function

import _dfhip
import _fieldmlp
import _gridencoder
from gridencoder.grid import _parts


def eligible(encoder, layers, x):
    if not (x.is_cuda and torch.is_autocast_enabled("cuda")):
        return False
    if torch.get_autocast_dtype("cuda") != torch.float16:
        return False
    if encoder.num_levels != 16 or encoder.level_dim != 2 or encoder.input_dim != 3:
        return False
    if len(layers) != 3 or layers[0].bias is None:
        return False
    shapes = [tuple(l.weight.shape) for l in layers]
    return shapes == [(64, 32), (64, 64), (4, 64)]


class _GridField(Function):
    @staticmethod
    def forward(ctx, x, bound, embeddings, offsets, meta, *weights):
        """x [M, 3] in [-bound, bound] f32 -> sigma [M] f32, albedo [M, 3] f16."""
        S, H, gridtype, align = meta
        x = x.contiguous().float()
        M = x.shape[0]
        x01 = ((x + bound) / (2 * bound)).contiguous()
        table = embeddings.to(torch.half).contiguous()
        rows = table.shape[0]
        L, C = offsets.shape[0] - 1, table.shape[1]
        enc = torch.empty(M, L * C, device=x.device, dtype=torch.half)
        nbytes = M * (12 + L * C * 2) + table.numel() * 2
        with _dfhip.timed("grid_encode_forward", nbytes):
            _gridencoder.grid_encode_forward_blc(x01, table, offsets, enc, M, 3, C, L, S, H, None,
                                                 gridtype, align)
        sigma = torch.empty(M, device=x.device, dtype=torch.float32)
        albedo = torch.empty(M, 3, device=x.device, dtype=torch.half)
        ws = [w.detach().float().contiguous() for w in weights]
        with _dfhip.timed("field_mlp_forward", M * (64 + 12 + 4 + 6)):
            _fieldmlp.field_mlp_forward(enc, x, ws, sigma, albedo)
        ctx.save_for_backward(x, x01, enc, offsets, *ws)
        ctx.meta = (S, H, gridtype, align, rows, L, C)
        return sigma, albedo

    @staticmethod
    def backward(ctx, grad_sigma, grad_albedo):
        x, x01, enc, offsets, *ws = ctx.saved_tensors
        S, H, gridtype, align, rows, L, C = ctx.meta
        M = x.shape[0]
        dev = x.device
        if grad_sigma is None:
            grad_sigma = torch.zeros(M, device=dev)
        if grad_albedo is None:
            grad_albedo = torch.zeros(M, 3, device=dev, dtype=torch.half)
        grad_sigma = grad_sigma.float().contiguous()
        grad_albedo = grad_albedo.contiguous()
        d_enc = torch.empty(L, M, C, device=dev, dtype=torch.half)
        parts = _fieldmlp.backward_parts(M) if M else 1
        partial = torch.empty(parts * _fieldmlp.params_count(), device=dev)
        grads = [torch.empty_like(w) for w in ws]
        with _dfhip.timed("field_mlp_backward", M * (64 + 12 + 4 + 6 + 64)):
            _fieldmlp.field_mlp_backward(enc, x, ws, grad_sigma, grad_albedo, d_enc, partial,
                                         grads)
        grad_emb = None
        if ctx.needs_input_grad[2]:
            gparts = _parts(rows, C)
            gpartial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, C, gparts),
                                   device=dev)
            grad_emb = torch.empty(rows, C, device=dev, dtype=torch.float32)
            nbytes = M * (12 + L * C * 2) + 4 * rows * C
            with _dfhip.timed("grid_encode_backward", nbytes):
                _gridencoder.grid_encode_backward_sliced(d_enc, x01, offsets, grad_emb, rows, M, 3,
                                                         C, L, S, H, gridtype, align, gpartial,
                                                         gparts)
        return (None, None, grad_emb, None, None, *grads)


def grid_field(x, bound, encoder, layers):
    """sigma [M] (f32), albedo [M, 3] (f16) of the grid field at x [M, 3]."""
    meta = (float(np.log2(encoder.per_level_scale)), int(encoder.base_resolution),
            encoder.gridtype_id, bool(encoder.align_corners))
    weights = []
    for lin in layers:
        weights += [lin.weight, lin.bias]
    return _GridField.apply(x, bound, encoder.embeddings, encoder.offsets, meta, *weights)
