"""Native fused field head (csrc/fieldmlp.hip): the grid NeRF's sigma MLP
32 -> 64 -> 64 -> 4 with trunc_exp density + Gaussian blob and sigmoid albedo
(reference nerf/network_grid.py:13-32,72-87), forward and backward, on MFMA.
No reference pybind counterpart: the reference runs this as torch ops."""
import torch

import _dfhip as _d
from _dfhip import call, checked, ptr, stream

IN, HIDDEN, OUT = 32, 64, 4


def params_count():
    return int(_d.load().dfhip_field_mlp_params())


def backward_parts(M):
    return int(_d.load().dfhip_field_mlp_backward_parts(M))


def _f32(t, what):
    checked(t, what)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{what} must be a float32 tensor")


def _weights(ws):
    if len(ws) != 6:
        raise RuntimeError("expected (w1, b1, w2, b2, w3, b3)")
    shapes = [(HIDDEN, IN), (HIDDEN,), (HIDDEN, HIDDEN), (HIDDEN,), (OUT, HIDDEN), (OUT,)]
    for i, (w, shp) in enumerate(zip(ws, shapes)):
        _f32(w, f"param{i}")
        if tuple(w.shape) != shp:
            raise RuntimeError(f"param{i} must have shape {shp}, got {tuple(w.shape)}")
    return [ptr(w) for w in ws]


def field_mlp_forward(enc, xyz, weights, sigma, rgb):
    """enc [M, 32] f16, xyz [M, 3] f32 -> sigma [M] f32, rgb [M, 3] (f16 or f32)."""
    M = enc.shape[0]
    checked(enc, "enc")
    if enc.dtype != torch.float16 or enc.shape[1] != IN:
        raise RuntimeError("enc must be a [M, 32] float16 tensor")
    _f32(xyz, "xyz")
    _f32(sigma, "sigma")
    checked(rgb, "rgb")
    call("dfhip_field_mlp_forward", ptr(enc), ptr(xyz), *_weights(weights), ptr(sigma), ptr(rgb),
         _d.dtype_code(rgb, "rgb"), M, stream())


def field_mlp_backward(enc, xyz, weights, grad_sigma, grad_rgb, d_enc_lbc, partial, grads,
                       accumulate=False):
    """grads: six f32 tensors shaped like the weights (overwritten, or added
    into with accumulate).  d_enc_lbc: [16, M, 2] f16.  partial:
    backward_parts(M) * params_count() f32 scratch."""
    M = enc.shape[0]
    for t, n in ((enc, "enc"), (grad_rgb, "grad_rgb"), (d_enc_lbc, "d_enc")):
        checked(t, n)
    _f32(xyz, "xyz")
    _f32(grad_sigma, "grad_sigma")
    _f32(partial, "partial")
    gp = _weights(grads)
    call("dfhip_field_mlp_backward", ptr(enc), ptr(xyz), *_weights(weights), ptr(grad_sigma),
         ptr(grad_rgb), _d.dtype_code(grad_rgb, "grad_rgb"), M, ptr(d_enc_lbc), ptr(partial),
         backward_parts(M) if M else 1, *gp, int(bool(accumulate)), stream())


# ---- the MLP module alone (network_grid.py:13-32), no heads

def mlp_forward(x, weights, out, m_dev=None):
    """x [cap, 32] f16 / bf16 -> out [cap, 4] (same dtype): the sigma_net
    MLP under autocast on MFMA.  Rows [m_dev[0], cap) of out are zeros when
    m_dev (int32 device live-row count) is given."""
    checked(x, "x")
    checked(out, "out")
    if x.dtype not in (torch.float16, torch.bfloat16) or x.dim() != 2 or x.shape[1] != IN:
        raise RuntimeError("x must be a [M, 32] float16 / bfloat16 tensor")
    if out.dtype != x.dtype or tuple(out.shape) != (x.shape[0], OUT):
        raise RuntimeError("out must be [M, 4] of x's dtype")
    if m_dev is not None:
        checked(m_dev, "m_dev", "int")
    call("dfhip_mlp_forward", _d.dtype_code(x, "x"), ptr(x), *_weights(weights), ptr(out),
         x.shape[0], ptr(m_dev), stream())


def mlp_backward(x, weights, dh, dx, partial, grads, m_dev=None, accumulate=False):
    """dh [cap, 4] (x's dtype) -> dx [cap, 32] (rows past m_dev[0] zero) and the
    six f32 weight gradients (overwritten, or added into with accumulate);
    partial: backward_parts(cap) * params_count() f32 scratch."""
    cap = x.shape[0]
    for t, n in ((x, "x"), (dh, "dh"), (dx, "dx")):
        checked(t, n)
        if t.dtype != x.dtype:
            raise RuntimeError(f"{n} must have x's dtype")
    if tuple(dh.shape) != (cap, OUT) or tuple(dx.shape) != (cap, IN):
        raise RuntimeError("dh must be [M, 4] and dx [M, 32]")
    _f32(partial, "partial")
    if m_dev is not None:
        checked(m_dev, "m_dev", "int")
    gp = _weights(grads)
    call("dfhip_mlp_backward", _d.dtype_code(x, "x"), ptr(x), *_weights(weights), ptr(dh), cap,
         ptr(m_dev), ptr(dx), ptr(partial), backward_parts(cap) if cap else 1, *gp,
         int(bool(accumulate)), stream())


# ---- fused grid field (encoding + MLP in one kernel; device-side sample count)

def grid_quads(embeddings, offsets, S, H, gridtype, align_corners, table, quads):
    """The autocast cast of the f32 embeddings [rows, 2] into `table` (f16 or
    bf16, [rows, 2]) and its corner quads into `quads` ([rows, 4] int32) for
    grid_field_forward(..., quads=quads)."""
    _f32(embeddings, "embeddings")
    checked(table, "table")
    checked(quads, "quads", "int")
    checked(offsets, "offsets", "int")
    rows = embeddings.shape[0]
    if table.dtype not in (torch.float16, torch.bfloat16) or tuple(table.shape) != (rows, 2) \
            or tuple(embeddings.shape) != (rows, 2):
        raise RuntimeError("embeddings [rows, 2] f32 and table [rows, 2] f16 / bf16 expected")
    if quads.dtype != torch.int32 or tuple(quads.shape) != (rows, 4):
        raise RuntimeError("quads must be a [rows, 4] int32 tensor")
    elem = _d.BF16 if table.dtype == torch.bfloat16 else _d.F16
    call("dfhip_grid_quads", elem, ptr(embeddings), ptr(offsets), offsets.shape[0] - 1, float(S),
         int(H), int(gridtype), int(bool(align_corners)), rows, ptr(table), ptr(quads), stream())


def grid_field_forward(xyz, bound, table, offsets, S, H, gridtype, align_corners, weights, enc,
                       sigma, rgb, m_dev=None,
                       quads=None):
    """xyz [cap, 3] f32 in [-bound, bound]; table [rows, 2] f16 (fp16 autocast,
    the reference's -O) or bf16 (the C5 bf16 option: features and activations
    bf16 too); offsets [17] int32.  Writes sigma [cap] f32, rgb [cap, 3] (the
    table's dtype or f32) and, when given, enc [cap, 32] in the table's dtype
    (permuted feature order, for grid_field_backward).  Only rows
    [0, m_dev[0]) are computed when m_dev (int32 device tensor) is given."""
    cap = xyz.shape[0]
    _f32(xyz, "xyz")
    checked(table, "table")
    if table.dtype not in (torch.float16, torch.bfloat16) or table.dim() != 2 or \
            table.shape[1] != 2:
        raise RuntimeError("table must be a [rows, 2] float16 or bfloat16 tensor")
    if enc is not None and enc.dtype != table.dtype:
        raise RuntimeError("enc must have the table's dtype")
    checked(offsets, "offsets", "int")
    _f32(sigma, "sigma")
    checked(rgb, "rgb")
    if enc is not None:
        checked(enc, "enc")
    if m_dev is not None:
        checked(m_dev, "m_dev", "int")
    if quads is not None:
        checked(quads, "quads", "int")
        if quads.dtype != torch.int32 or tuple(quads.shape) != (table.shape[0], 4):
            raise RuntimeError("quads must be a [rows, 4] int32 tensor (rows = table rows)")
        elem = _d.BF16 if table.dtype == torch.bfloat16 else _d.F16
        call("dfhip_grid_field_forward_quads", elem, ptr(xyz), float(bound), ptr(table),
             ptr(quads), ptr(offsets), offsets.shape[0] - 1, float(S), int(H), int(gridtype),
             int(bool(align_corners)), *_weights(weights), ptr(enc), ptr(sigma), ptr(rgb),
             _d.dtype_code(rgb, "rgb"), cap, ptr(m_dev), stream())
        return
    fn = "dfhip_grid_field_forward_bf16" if table.dtype == torch.bfloat16 else \
        "dfhip_grid_field_forward"
    call(fn, ptr(xyz), float(bound), ptr(table), ptr(offsets),
         offsets.shape[0] - 1, float(S), int(H), int(gridtype), int(bool(align_corners)),
         *_weights(weights), ptr(enc), ptr(sigma), ptr(rgb), _d.dtype_code(rgb, "rgb"), cap,
         ptr(m_dev), stream())


def grid_field_backward(enc, xyz, bound, weights, grad_sigma, grad_rgb, d_enc_lbc, mlp_partial,
                        grads, offsets, total_rows, S, H, gridtype, align_corners,
                        grad_embeddings, grid_partial, grid_parts, m_dev=None, accumulate=False):
    """accumulate: add into grads (and grad_embeddings) instead of overwriting
    (the second backward of the reference's two-pass step)."""
    cap = xyz.shape[0]
    for t, n in ((enc, "enc"), (grad_rgb, "grad_rgb"), (d_enc_lbc, "d_enc")):
        checked(t, n)
    _f32(xyz, "xyz")
    _f32(grad_sigma, "grad_sigma")
    _f32(mlp_partial, "mlp_partial")
    if grad_embeddings is not None:
        _f32(grad_embeddings, "grad_embeddings")
        _f32(grid_partial, "grid_partial")
    if m_dev is not None:
        checked(m_dev, "m_dev", "int")
    gp = _weights(grads)
    if enc.dtype == torch.bfloat16:
        # bf16 field: the embedding gradient is the binned backward's (bf16 grads)
        if grad_embeddings is not None:
            raise RuntimeError("bf16 field: grad_embeddings must be None (use the binned "
                               "embedding backward on d_enc_lbc)")
        if d_enc_lbc.dtype != torch.bfloat16:
            raise RuntimeError("bf16 field: d_enc must be bfloat16")
        call("dfhip_grid_field_backward_bf16", ptr(enc), ptr(xyz), float(bound),
             *_weights(weights), ptr(grad_sigma), ptr(grad_rgb),
             _d.dtype_code(grad_rgb, "grad_rgb"), cap, ptr(m_dev), ptr(d_enc_lbc),
             ptr(mlp_partial), backward_parts(cap) if cap else 1, *gp, int(bool(accumulate)),
             stream())
        return
    call("dfhip_grid_field_backward_accumulate" if accumulate else "dfhip_grid_field_backward",
         ptr(enc), ptr(xyz), float(bound), *_weights(weights),
         ptr(grad_sigma), ptr(grad_rgb), _d.dtype_code(grad_rgb, "grad_rgb"), cap, ptr(m_dev),
         ptr(d_enc_lbc), ptr(mlp_partial), backward_parts(cap) if cap else 1, *gp,
         ptr(offsets), int(total_rows), offsets.shape[0] - 1, float(S), int(H), int(gridtype),
         int(bool(align_corners)), ptr(grad_embeddings), ptr(grid_partial), int(grid_parts),
         stream())


# ---- fused inference render (march + field + composite, persistent queue)

def render_ray_order(rays_o, rays_d, chunk_log2=6, cost=None, order=None, occ=None, tile_w=0):
    """Queue order of the fused render (csrc/render.hip k_chunk_cost +
    k_chunk_sort): the chunks of 2^chunk_log2 consecutive rays (tile_w > 0:
    8 x 8 pixel tiles of a row-major image tile_w wide) by ascending
    summed squared distance of their lines from the origin.  Returns the
    [ceil(N / 2^chunk_log2)] int32 order (cost: f32 scratch of that size).
    occ = (nears, fars, bitfield, bound, C, H, max_steps): cost from the
    occupancy grid instead (dfhip_render_ray_order_occ)."""
    n = rays_o.shape[0]
    _f32(rays_o, "rays_o")
    _f32(rays_d, "rays_d")
    if tuple(rays_o.shape) != (n, 3) or tuple(rays_d.shape) != (n, 3):
        raise RuntimeError("rays_o and rays_d must be [N, 3]")
    nc = -(-n // (1 << chunk_log2))
    if cost is None:
        cost = torch.empty(nc, dtype=torch.float32, device=rays_o.device)
    if order is None:
        order = torch.empty(nc, dtype=torch.int32, device=rays_o.device)
    _f32(cost, "cost")
    checked(order, "order", "int")
    if cost.numel() < nc or order.numel() < nc:
        raise RuntimeError("cost / order must hold ceil(N / 2^chunk_log2) values")
    if occ is None:
        call("dfhip_render_ray_order", ptr(rays_o), ptr(rays_d), n, int(chunk_log2), int(tile_w),
             ptr(cost),
             ptr(order), stream())
    else:  # (nears, fars, bitfield, bound, C, H, max_steps): occupancy cost
        nears, fars, bitfield, bound, C, H, max_steps = occ
        _f32(nears, "nears")
        _f32(fars, "fars")
        checked(bitfield, "bitfield", "u8")
        if tuple(nears.shape) != (n,) or tuple(fars.shape) != (n,):
            raise RuntimeError("nears / fars must be [N]")
        if bitfield.numel() * 8 < C * H ** 3:
            raise RuntimeError("bitfield is smaller than C * H^3 / 8 bytes")
        call("dfhip_render_ray_order_occ", ptr(rays_o), ptr(rays_d), ptr(nears), ptr(fars),
             ptr(bitfield), float(bound), int(C), int(H), int(max_steps), n, int(chunk_log2),
             int(tile_w),
             ptr(cost), ptr(order), stream())
    return order


def render_rays_infer(rays_o, rays_d, nears, fars, noises, bound, dt_gamma, max_steps, C, H,
                      bitfield, T_thresh, table, offsets, S, base_res, gridtype, align_corners,
                      weights, weights_sum, depth, image, work, quads=None, prof=None,
                      order=None, chunk_log2=6, tile_w=0):
    """Inference render of N rays in one launch (csrc/render.hip; reference
    nerf/renderer.py:496-532).  rays_o/rays_d [N, 3] f32, nears/fars [N] f32,
    noises [N] f32 or None, bitfield u8, table [rows, 2] f16, offsets int32.
    Writes weights_sum [N], depth [N], image [N, 3] f32; work: [4] int32
    scratch whose words 1, 2 hold the evaluated sample count afterwards;
    quads: the table's corner quads ([rows, 4] int32, grid_quads) or None.
    prof: [16 + 16 W] int64 device tensor receiving the kernel's per-wave phase
    cycles and its wall-clock drain profile (dfhip_render_rays_infer_prof:
    [6], [7] set to -1, the rest to 0 by the caller; tools only) or None.
    order: [ceil(N / 2^chunk_log2)] int32 device permutation of the chunks
    of 2^chunk_log2 consecutive rays (tile_w > 0: 8 x 8 pixel tiles of a
    row-major image tile_w wide, as given to render_ray_order), the queue's
    order (render_ray_order; taken in mirrored halves, see
    dfhip_render_rays_infer_ordered; outputs are per ray, so identical), or
    None for pixel order."""
    n = rays_o.shape[0]
    for t, what in ((rays_o, "rays_o"), (rays_d, "rays_d"), (nears, "nears"), (fars, "fars"),
                    (weights_sum, "weights_sum"), (depth, "depth"), (image, "image")):
        _f32(t, what)
    if tuple(rays_d.shape) != (n, 3) or tuple(rays_o.shape) != (n, 3):
        raise RuntimeError("rays_o and rays_d must be [N, 3]")
    for t, what, shp in ((nears, "nears", (n,)), (fars, "fars", (n,)),
                         (weights_sum, "weights_sum", (n,)), (depth, "depth", (n,)),
                         (image, "image", (n, 3))):
        if tuple(t.shape) != shp:
            raise RuntimeError(f"{what} must have shape {shp}, got {tuple(t.shape)}")
    if noises is not None:
        _f32(noises, "noises")
        if tuple(noises.shape) != (n,):
            raise RuntimeError("noises must be [N]")
    checked(bitfield, "bitfield", "u8")
    if bitfield.numel() * 8 < C * H ** 3:
        raise RuntimeError("bitfield is smaller than C * H^3 / 8 bytes")
    checked(table, "table")
    if table.dtype != torch.float16 or table.dim() != 2 or table.shape[1] != 2:
        raise RuntimeError("table must be a [rows, 2] float16 tensor")
    checked(offsets, "offsets", "int")
    checked(work, "work", "int")
    if work.numel() < 4:
        raise RuntimeError("work must hold 4 int32")
    if quads is not None:
        checked(quads, "quads", "int")
        if tuple(quads.shape) != (table.shape[0], 4):
            raise RuntimeError("quads must be [rows, 4] int32 (grid_quads of the table)")
    args = (n, ptr(rays_o), ptr(rays_d), ptr(nears), ptr(fars), ptr(noises), float(bound),
            float(dt_gamma), int(max_steps), int(C), int(H), ptr(bitfield), float(T_thresh),
            ptr(table), ptr(offsets), offsets.shape[0] - 1, float(S), int(base_res),
            int(gridtype), int(bool(align_corners)), *_weights(weights), ptr(weights_sum),
            ptr(depth), ptr(image), ptr(work), ptr(quads))
    if prof is not None:
        checked(prof, "prof", "i64")
        if prof.numel() < 16 or prof.numel() < 16 + 16 * int(prof[10]):
            raise RuntimeError("prof must hold 16 + 16 prof[10] int64 values")
    if order is not None:
        checked(order, "order", "int")
        if tuple(order.shape) != (-(-n // (1 << chunk_log2)),):
            raise RuntimeError("order must be [ceil(N / 2^chunk_log2)] int32")
        call("dfhip_render_rays_infer_ordered", *args, ptr(order), int(chunk_log2), int(tile_w),
             ptr(prof), stream())
    elif prof is None:
        call("dfhip_render_rays_infer", *args, stream())
    else:
        call("dfhip_render_rays_infer_prof", *args, ptr(prof), stream())
