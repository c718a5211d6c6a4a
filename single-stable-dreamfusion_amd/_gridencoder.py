"""`_gridencoder` backend module: the reference pybind11 surface
(gridencoder/src/bindings.cpp, gridencoder.h:12-13) over the gfx950 C-ABI,
plus the native [B, L*C]-layout entry points.  Checks mirror
gridencoder.cu:425-441 (CHECK_CUDA / CHECK_CONTIGUOUS / dtype) and raise
RuntimeError."""
import ctypes

import _dfhip as _d
from _dfhip import call, ptr, stream, checked


def _common(inputs, embeddings, offsets):
    checked(inputs, "inputs")
    if inputs.dtype.itemsize != 4 or not inputs.is_floating_point():
        raise RuntimeError("inputs must be a float32 tensor")
    checked(embeddings, "embeddings")
    checked(offsets, "offsets", "int")
    return _d.dtype_code(embeddings, "embeddings")


def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx, gridtype,
                        align_corners):
    dt = _common(inputs, embeddings, offsets)
    checked(outputs, "outputs")
    call("dfhip_grid_encode_forward", dt, ptr(inputs), ptr(embeddings), ptr(offsets), ptr(outputs),
         B, D, C, L, S, H, ptr(dy_dx), gridtype, int(bool(align_corners)), stream())


def grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S, H,
                         dy_dx, grad_inputs, gridtype, align_corners):
    """gridencoder.cu:449-479: ADDS d(outputs)/d(embeddings) . grad into
    grad_embeddings (the caller zero-fills it, grid.py:72), grad [L, B, C].
    Without an input gradient (dy_dx None, the NeRF path) the sum comes from
    the binned owner-computes walk (exact f64 sums rounded to f32 once, then
    added into grad_embeddings in its dtype: f16 under autocast, where the
    reference rounds every atomic add to half); with dy_dx, or a shape the
    walk does not take, from the reference's atomic scatter."""
    import torch
    from gridencoder.grid import binned_eligible, binned_embedding_grad, host_offsets
    dt = _common(inputs, embeddings, offsets)
    checked(grad, "grad")
    checked(grad_embeddings, "grad_embeddings")
    if (dy_dx is None and grad_inputs is None and binned_eligible(D, C, grad.dtype)
            and grad.dtype == embeddings.dtype and grad_embeddings.dtype in (torch.float16,
                                                                            torch.float32)):
        if B == 0:
            return
        offs_h = host_offsets(offsets)
        f32 = grad_embeddings.dtype == torch.float32
        out = binned_embedding_grad(grad, inputs, 0.0, offsets, offs_h, B, None, C, L, S, H,
                                    gridtype, align_corners,
                                    out=grad_embeddings if f32 else None, accumulate=f32)
        if not f32:
            grad_embeddings.add_(out.to(grad_embeddings.dtype))
        return
    call("dfhip_grid_encode_backward", dt, ptr(grad), ptr(inputs), ptr(embeddings), ptr(offsets),
         ptr(grad_embeddings), B, D, C, L, S, H, ptr(dy_dx), ptr(grad_inputs), gridtype,
         int(bool(align_corners)), stream())


def grid_encode_forward_blc(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx, gridtype,
                            align_corners):
    dt = _common(inputs, embeddings, offsets)
    checked(outputs, "outputs")
    call("dfhip_grid_encode_forward_blc", dt, ptr(inputs), ptr(embeddings), ptr(offsets),
         ptr(outputs), B, D, C, L, S, H, ptr(dy_dx), gridtype, int(bool(align_corners)), stream())


def grid_encode_forward_dyn(inputs, bound, embeddings, offsets, outputs, B, m_dev, D, C, L, S, H,
                            dy_dx, gridtype, align_corners):
    """grid_encode_forward_blc over a capacity-sized batch: rows [0, m_dev[0])
    encoded, the rest zero; raw inputs in [-bound, bound] when bound > 0."""
    dt = _common(inputs, embeddings, offsets)
    checked(outputs, "outputs")
    if m_dev is not None:
        checked(m_dev, "m_dev", "int")
    call("dfhip_grid_encode_forward_dyn", dt, ptr(inputs), float(bound), ptr(embeddings),
         ptr(offsets), ptr(outputs), B, ptr(m_dev), D, C, L, S, H, ptr(dy_dx), gridtype,
         int(bool(align_corners)), stream())


def grid_encode_backward_blc(grad, inputs, offsets, grad_embeddings, B, D, C, L, S, H, dy_dx,
                             grad_inputs, gridtype, align_corners):
    checked(grad, "grad")
    checked(inputs, "inputs")
    checked(offsets, "offsets", "int")
    checked(grad_embeddings, "grad_embeddings")
    call("dfhip_grid_encode_backward_blc", _d.dtype_code(grad, "grad"),
         _d.dtype_code(grad_embeddings, "grad_embeddings"), ptr(grad), ptr(inputs), ptr(offsets),
         ptr(grad_embeddings), B, D, C, L, S, H, ptr(dy_dx), ptr(grad_inputs), gridtype,
         int(bool(align_corners)), stream())


# ---- native sliced backward (LDS-privatised, no global atomics; see dfhip.h)

def grid_grad_blc_to_lbc(grad, out, B, L, C):
    """[B, L*C] -> [L, B, C] (same dtype, contiguous out)."""
    checked(grad, "grad")
    checked(out, "out")
    call("dfhip_grid_grad_blc_to_lbc", _d.dtype_code(grad, "grad"), ptr(grad), ptr(out), B, L, C,
         stream())


def grid_backward_default_parts(total_rows, C):
    return int(_d.load().dfhip_grid_backward_default_parts(total_rows, C))


def grid_backward_partial_floats(total_rows, C, parts):
    return int(_d.load().dfhip_grid_backward_partial_floats(total_rows, C, parts))


def grid_encode_backward_sliced(grad_lbc, inputs, offsets, grad_embeddings, total_rows, B, D, C, L,
                                S, H, gridtype, align_corners, partial, parts, accumulate=False):
    checked(grad_lbc, "grad")
    checked(inputs, "inputs")
    checked(offsets, "offsets", "int")
    checked(grad_embeddings, "grad_embeddings")
    checked(partial, "partial")
    call("dfhip_grid_encode_backward_sliced", _d.dtype_code(grad_lbc, "grad"),
         _d.dtype_code(grad_embeddings, "grad_embeddings"), ptr(grad_lbc), ptr(inputs),
         ptr(offsets), ptr(grad_embeddings), total_rows, B, D, C, L, S, H, gridtype,
         int(bool(align_corners)), ptr(partial), parts, int(bool(accumulate)), stream())


def grid_encode_backward_sliced_dyn(grad_lbc, inputs, bound, offsets, grad_embeddings, total_rows,
                                    B, m_dev, D, C, L, S, H, gridtype, align_corners, partial,
                                    parts, accumulate=False):
    """Capacity form: grad_lbc [L, B, C] with B the capacity; rows [0, m_dev[0])
    walked; inputs raw positions in [-bound, bound] when bound > 0."""
    checked(grad_lbc, "grad")
    checked(inputs, "inputs")
    checked(offsets, "offsets", "int")
    checked(grad_embeddings, "grad_embeddings")
    checked(partial, "partial")
    if m_dev is not None:
        checked(m_dev, "m_dev", "int")
    call("dfhip_grid_encode_backward_sliced_dyn", _d.dtype_code(grad_lbc, "grad"),
         _d.dtype_code(grad_embeddings, "grad_embeddings"), ptr(grad_lbc), ptr(inputs),
         float(bound), ptr(offsets), ptr(grad_embeddings), total_rows, B, ptr(m_dev), D, C, L, S,
         H, gridtype, int(bool(align_corners)), ptr(partial), parts, int(bool(accumulate)),
         stream())


# ---- binned owner-computes backward (csrc/gridbin.hip; see dfhip.h)

class BinnedOpts(ctypes.Structure):
    """dfhip_binned_opts: per-call A/B and test switches of the binned
    backward (fields < 0 keep the library default; see include/dfhip.h)."""
    _fields_ = [("walk_mode", ctypes.c_int32), ("fast_bin", ctypes.c_int32),
                ("walk_groups_per_cu", ctypes.c_int32), ("lane_perm", ctypes.c_int32),
                ("kept_clean", ctypes.c_int32), ("trace", ctypes.c_void_p)]

    def __init__(self, walk_mode=-1, fast_bin=-1, walk_groups_per_cu=0, lane_perm=-1,
                 trace=None, kept_clean=0):
        super().__init__(int(walk_mode), int(fast_bin), int(walk_groups_per_cu), int(lane_perm),
                         int(kept_clean), None if trace is None else ptr(trace))


def _opts_ref(opts):
    return None if opts is None else ctypes.byref(opts)


def grid_backward_binned_tile(opts=None, group=1):
    """Samples per binning tile (id slots per (tile, slice) segment)."""
    return int(_d.load().dfhip_grid_backward_binned_tile(int(group), _opts_ref(opts)))


def grid_backward_binned_scratch(cap, offsets_host, L, C, opts=None, group=1):
    """(entries u32, counts u32, partial f32) element counts for capacity cap
    (samples, or stencil groups with group=7; opts: the BinnedOpts the
    launches will use).  Host only."""
    import numpy as np
    off = np.ascontiguousarray(offsets_host, dtype=np.int32)
    e, c, p = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    call("dfhip_grid_backward_binned_scratch_opts", int(cap), off.ctypes.data, int(L), int(C),
         int(group), _opts_ref(opts), ctypes.byref(e), ctypes.byref(c), ctypes.byref(p))
    return int(e.value), int(c.value), int(p.value)


def grid_encode_backward_binned(*args, **kw):
    """Validate and launch once (see binned_launcher)."""
    binned_launcher(*args, **kw)()


def binned_launcher(grad_lbc, inputs, bound, offsets, offsets_host, grad_embeddings,
                    B, m_dev, D, C, L, S, H, gridtype, align_corners, entries, counts,
                    partial, accumulate=False, phase=3, stencil_eps=None, opts=None):
    """grad_lbc [L, B, C] (B = capacity), inputs [B, D] raw positions in
    [-bound, bound] (bound > 0) or [0, 1] (bound = 0); rows [0, m_dev[0]) walked
    when m_dev is given.  grad_embeddings [rows, C] f32 is overwritten (or
    added into with accumulate).  stencil_eps: finite-difference stencil
    groups of 7 (dfhip_grid_encode_backward_binned_stencil): grad_lbc is
    [L, 7 B, C], inputs / B / m_dev count samples, row 7 g + a is point a of
    sample g's stencil.  opts: BinnedOpts of this call (None = defaults; the
    scratch must be sized with the same opts)."""
    import numpy as np
    checked(grad_lbc, "grad")
    checked(inputs, "inputs")
    checked(offsets, "offsets", "int")
    checked(grad_embeddings, "grad_embeddings")
    if grad_embeddings.dtype.itemsize != 4:
        raise RuntimeError("grad_embeddings must be float32")
    checked(entries, "entries", "int")
    checked(counts, "counts", "int")
    checked(partial, "partial")
    if m_dev is not None:
        checked(m_dev, "m_dev", "int")
    off = np.ascontiguousarray(offsets_host, dtype=np.int32)
    if phase not in (1, 2, 3):
        raise RuntimeError("phase must be 1 (bin), 2 (walk + sum) or 3 (both)")
    head = (int(phase), _d.dtype_code(grad_lbc, "grad"), ptr(grad_lbc), ptr(inputs), float(bound),
            ptr(offsets), off.ctypes.data, ptr(grad_embeddings), int(B), ptr(m_dev), int(D),
            int(C), int(L), float(S), int(H), int(gridtype), int(bool(align_corners)))
    tail = (ptr(entries), ptr(counts), ptr(partial), int(bool(accumulate)))
    keep = (grad_lbc, inputs, offsets, off, grad_embeddings, m_dev, entries, counts, partial,
            opts)
    if stencil_eps is not None and (grad_lbc.shape[1] < 7 * int(B) or inputs.shape[0] < int(B)):
        raise RuntimeError("stencil groups: grad_lbc must hold 7 B rows per level and "
                           "inputs B samples")
    group = (1, 0.0) if stencil_eps is None else (7, float(stencil_eps))
    name, args = ("dfhip_grid_encode_backward_binned_opts",
                  head + group + tail + (_opts_ref(opts),))

    def launch(_keep=keep):
        """Launch on the current stream with the validated, pre-marshalled
        arguments (the graph-replayed step calls this every step)."""
        call(name, *args, stream())
    return launch
