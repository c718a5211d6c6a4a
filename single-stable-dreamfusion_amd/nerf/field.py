"""Fused grid field: tiled-grid encoding + sigma MLP + density/albedo heads as
ONE autograd node on the native kernels (the reference's
network_grid.common_forward, nerf/network_grid.py:76-87, = GridEncoder ->
MLP -> trunc_exp(h0 + gaussian) / sigmoid(h[1:])).

Forward: dfhip_grid_field_forward — grid gather and MLP in one kernel, the
features kept (permuted order) for the backward.  Backward:
dfhip_grid_field_backward — MLP backward (recomputed from the features, the
feature gradient written straight into the [L, B, C] layout) then the sliced
embedding backward.  With `m_dev` (the march's device-side sample count)
only the live rows of capacity-sized buffers are processed, so the train
step needs no host round trip.  Used under fp16 autocast for the reference's
network shape (16 levels x 2 channels, 32 -> 64 -> 64 -> 4), and under bf16
autocast (the C5 option: the table, features and activations in bf16, the
embedding gradient by the binned backward); anything else runs the unfused
modules.
"""
import numpy as np
import torch
from torch.autograd import Function

import _dfhip
import _fieldmlp
import _gridencoder
from gridencoder.grid import _parts


# When a list, _GridField.backward appends (launch, grad_buffer) instead of
# launching the embedding backward (see defer_embedding_backward).
_deferred = None


class defer_embedding_backward:
    """Context: collect the fused field's embedding-gradient launches instead of
    running them inside the backward.  Used while capturing the train step in
    a HIP graph: the graph holds everything up to the feature gradients, and
    the embedding scatter (the step's largest kernel) is launched after each
    replay, timed on its stream like any eager launch."""

    def __enter__(self):
        global _deferred
        self.prev, _deferred = _deferred, []
        return _deferred

    def __exit__(self, *exc):
        global _deferred
        _deferred = self.prev
        return False


def eligible(encoder, layers, x):
    if not (x.is_cuda and torch.is_autocast_enabled("cuda")):
        return False
    if torch.get_autocast_dtype("cuda") not in (torch.float16, torch.bfloat16):
        return False
    if torch.get_autocast_dtype("cuda") == torch.bfloat16 and (
            getattr(encoder, "offsets_host", None) is None):
        return False  # bf16 feature gradients: binned embedding backward only
    if encoder.num_levels != 16 or encoder.level_dim != 2 or encoder.input_dim != 3:
        return False
    if len(layers) != 3 or layers[0].bias is None:
        return False
    shapes = [tuple(l.weight.shape) for l in layers]
    return shapes == [(64, 32), (64, 64), (4, 64)]


class _GridField(Function):
    @staticmethod
    def forward(ctx, x, bound, embeddings, offsets, meta, m_dev, *weights):
        """x [cap, 3] in [-bound, bound] f32 -> sigma [cap] f32, albedo [cap, 3]
        f16 (rows >= m_dev[0] untouched when m_dev is given)."""
        S, H, gridtype, align, offsets_host = meta
        x = x.contiguous().float()
        cap = x.shape[0]
        elem = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") \
            else torch.half  # f16 (fp16 autocast) or bf16 (bf16 autocast)
        table = embeddings.to(elem).contiguous()
        L, C = offsets.shape[0] - 1, table.shape[1]
        enc = torch.empty(cap, L * C, device=x.device, dtype=elem)
        sigma = torch.empty(cap, device=x.device, dtype=torch.float32)
        albedo = torch.empty(cap, 3, device=x.device, dtype=elem)
        ws = [w.detach().float().contiguous() for w in weights]
        # algorithmic bytes per sample: xyz + features out + sigma/albedo out,
        # plus the f16 table once (the gathers hit L2 / MALL)
        per, base = 12 + 64 + 4 + 6, table.numel() * 2
        with _dfhip.timed("grid_field_forward", base + (0 if m_dev is not None else cap * per),
                          m_dev, per):
            _fieldmlp.grid_field_forward(x, bound, table, offsets, S, H, gridtype, align, ws, enc,
                                         sigma, albedo, m_dev)
        ctx.save_for_backward(x, enc, offsets, m_dev, *ws)
        ctx.meta = (S, H, gridtype, align, table.shape[0], L, C, float(bound), offsets_host)
        return sigma, albedo

    @staticmethod
    def backward(ctx, grad_sigma, grad_albedo):
        x, enc, offsets, m_dev, *ws = ctx.saved_tensors
        S, H, gridtype, align, rows, L, C, bound, offsets_host = ctx.meta
        cap = x.shape[0]
        dev = x.device
        if grad_sigma is None:
            grad_sigma = torch.zeros(cap, device=dev)
        if grad_albedo is None:
            grad_albedo = torch.zeros(cap, 3, device=dev, dtype=enc.dtype)
        grad_sigma = grad_sigma.float().contiguous()
        grad_albedo = grad_albedo.to(enc.dtype).contiguous()
        d_enc = torch.empty(L, cap, C, device=dev, dtype=enc.dtype)
        mlp_partial = torch.empty((_fieldmlp.backward_parts(cap) if cap else 1)
                                  * _fieldmlp.params_count(), device=dev)
        grads = [torch.empty_like(w) for w in ws]
        grad_emb = gpartial = None
        gparts = _parts(rows, C)
        binned = offsets_host is not None
        if ctx.needs_input_grad[2]:
            grad_emb = torch.empty(rows, C, device=dev, dtype=torch.float32)
            if binned:
                ne, nc, npf = _gridencoder.grid_backward_binned_scratch(cap, offsets_host, L, C)
                scratch = (torch.empty(ne, device=dev, dtype=torch.int32),
                           torch.empty(nc, device=dev, dtype=torch.int32),
                           torch.empty(npf, device=dev))
            else:
                gpartial = torch.empty(_gridencoder.grid_backward_partial_floats(rows, C, gparts),
                                       device=dev)
        # MLP backward: features + positions + incoming grads in, feature grads out
        per = 64 + 12 + 4 + 6 + 64
        with _dfhip.timed("field_mlp_backward", 0 if m_dev is not None else cap * per, m_dev,
                          per):
            _fieldmlp.grid_field_backward(enc, x, bound, ws, grad_sigma, grad_albedo, d_enc,
                                          mlp_partial, grads, offsets, rows, S, H, gridtype,
                                          align, None, None, gparts, m_dev)
        if grad_emb is not None:
            launch = None
            if binned:
                launch = _gridencoder.binned_launcher(d_enc, x, bound, offsets, offsets_host,
                                                      grad_emb, cap, m_dev, 3, C, L, S, H,
                                                      gridtype, align, *scratch)

            def embedding_backward(grad_emb=grad_emb):
                # algorithmic bytes: per live sample its position and feature
                # grads, plus the table gradient once
                per = 12 + L * C * 2
                base, live = 4 * rows * C, m_dev
                if live is None:
                    base += cap * per
                with _dfhip.timed("grid_encode_backward", base, live, per):
                    if launch is not None:
                        launch()
                    else:
                        _gridencoder.grid_encode_backward_sliced_dyn(
                            d_enc, x, bound, offsets, grad_emb, rows, cap, m_dev, 3, C, L, S, H,
                            gridtype, align, gpartial, gparts)
                return grad_emb

            if _deferred is not None:
                # graph capture: the embedding scatter runs after the replay
                # (Trainer), the gradient lands in grad_emb, not via autograd
                _deferred.append((embedding_backward, grad_emb))
                grad_emb = None
            else:
                embedding_backward()
        return (None, None, grad_emb, None, None, None, *grads)


def grid_field(x, bound, encoder, layers, m_dev=None):
    """sigma [M] (f32), albedo [M, 3] (autocast dtype) of the grid field at x [M, 3].
    m_dev: optional int32 device tensor holding the live row count."""
    meta = (float(np.log2(encoder.per_level_scale)), int(encoder.base_resolution),
            encoder.gridtype_id, bool(encoder.align_corners),
            getattr(encoder, "offsets_host", None))
    weights = []
    for lin in layers:
        weights += [lin.weight, lin.bias]
    return _GridField.apply(x, bound, encoder.embeddings, encoder.offsets, meta, m_dev, *weights)
