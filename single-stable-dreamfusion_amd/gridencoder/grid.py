"""Multi-resolution grid encoder (mirror of reference gridencoder/grid.py).

Public surface identical to the reference: `grid_encode` (autograd Function)
and `GridEncoder(input_dim, num_levels, level_dim, per_level_scale,
base_resolution, log2_hashmap_size, desired_resolution, gridtype,
align_corners)` with the same parameter layout (`offsets`, `embeddings`,
grid.py:91-133) and the same autocast rule (half embeddings when C is even,
grid.py:38-39).

GPU-side differences (invisible to callers):

* outputs are produced directly in the [B, L*C] layout the caller consumes
  (no [L, B, C] buffer + permute copy, grid.py:42,52,70);
* the embedding backward is the binned owner-computes walk
  (csrc/gridbin.hip: exact f64 sums, no global atomics, deterministic) in
  place of the reference's half2 atomics (gridencoder.cu:226-313); the
  reference's atomic scatter stays available as `GridEncoder.backward_mode =
  "atomic"` and is taken when the input gradient is requested (dy_dx);
* capacity-sized batches: inputs that carry a device live-row count
  (`raymarching.live_rows`, the device-count march) are encoded up to that
  count only — rows past it come out as zeros — and the backward walks only
  those rows; GridEncoder passes the raw positions and `bound` to the kernels
  (the map (x + bound) / (2 bound) of grid.py:142 is done there, bit for bit).
"""
import numpy as np
import torch
import torch.nn as nn
from torch.autograd import Function
from torch.amp import custom_bwd, custom_fwd

import _dfhip
import _gridencoder as _backend

_gridtype_to_id = {"hash": 0, "tiled": 1}

# attribute name of the device live-row count on capacity-sized tensors
# (raymarching.march_rays_train_dev sets it; raymarching.live_rows reads it)
_LIVE_ROWS_ATTR = "_dfhip_live_rows"

_parts_cache = {}


def _parts(total_rows, C):
    key = (total_rows, C)
    if key not in _parts_cache:
        _parts_cache[key] = _backend.grid_backward_default_parts(total_rows, C)
    return _parts_cache[key]


_host_offsets_cache = {}


def host_offsets(offsets):
    """Host copy of a level-offset tensor (the binned backward plans its slices
    on the host).  Cached per (storage, version): a copy per new tensor only."""
    key = (offsets.data_ptr(), offsets._version, offsets.numel(), str(offsets.device))
    got = _host_offsets_cache.get(key)
    if got is None:
        got = offsets.detach().to("cpu", torch.int32).numpy().copy()
        if len(_host_offsets_cache) > 64:
            _host_offsets_cache.clear()
        _host_offsets_cache[key] = got
    return got


def binned_eligible(D, C, grad_dtype):
    """The binned walk handles this shape / gradient dtype (gridbin.hip)."""
    if D != 3 or C not in (1, 2, 4):
        return False
    if grad_dtype == torch.bfloat16:
        return C == 2
    return grad_dtype in (torch.float16, torch.float32)


def binned_embedding_grad(grad_lbc, inputs, bound, offsets, offsets_host, B, m_dev, C, L, S, H,
                          gridtype, align_corners, out=None, accumulate=False):
    """grad_embeddings (f32 [rows, C]) of grad_lbc [L, B, C] through the binned
    owner-computes walk (scratch allocated here, from the caching allocator).
    inputs [B, 3]: raw positions when bound > 0, else in [0, 1]; rows
    [0, m_dev[0]) when m_dev is given."""
    rows = int(offsets_host[-1])
    dev = grad_lbc.device
    ne, nc, npf = _backend.grid_backward_binned_scratch(B, offsets_host, L, C)
    ent = torch.empty(ne, dtype=torch.int32, device=dev)
    cnt = torch.empty(nc, dtype=torch.int32, device=dev)
    part = torch.empty(npf, dtype=torch.float32, device=dev)
    if out is None:
        out = torch.empty(rows, C, dtype=torch.float32, device=dev)
    _backend.grid_encode_backward_binned(grad_lbc, inputs, float(bound), offsets, offsets_host,
                                         out, B, m_dev, 3, C, L, S, H, gridtype,
                                         bool(align_corners), ent, cnt, part, accumulate)
    return out


class _grid_encode(Function):
    @staticmethod
    @custom_fwd(device_type="cuda")
    def forward(ctx, inputs, embeddings, offsets, per_level_scale, base_resolution,
                calc_grad_inputs=False, gridtype=0, align_corners=False, offsets_host=None,
                bound=0.0, m_dev=None, backward_mode="binned"):
        """inputs [B, D] in [0, 1] (f32), embeddings [sum_l rows_l, C],
        offsets [L+1] int32 -> [B, L*C] (half under autocast when C is even).
        Past the reference's arguments (all optional): offsets_host (host
        copy of offsets), bound > 0 (inputs are raw positions in [-bound,
        bound]), m_dev (int32 device live-row count of a capacity-sized batch:
        rows past it come out zero and get no gradient), backward_mode
        ("binned" or the reference's "atomic")."""
        inputs = inputs.contiguous()
        B, D = inputs.shape
        L = offsets.shape[0] - 1
        C = embeddings.shape[1]
        S = float(np.log2(per_level_scale))
        H = int(base_resolution)
        table = embeddings
        if torch.is_autocast_enabled("cuda") and C % 2 == 0:
            table = embeddings.to(torch.half)
        table = table.contiguous()
        outputs = torch.empty(B, L * C, device=inputs.device, dtype=table.dtype)
        dy_dx = (torch.empty(B, L * D * C, device=inputs.device, dtype=table.dtype)
                 if calc_grad_inputs else None)
        es = table.element_size()
        # algorithmic bytes: inputs + outputs per sample, table once
        if m_dev is not None or bound > 0:
            with _dfhip.timed("grid_encode_forward", table.numel() * es, m_dev,
                              4 * D + L * C * es):
                _backend.grid_encode_forward_dyn(inputs, float(bound), table, offsets, outputs,
                                                 B, m_dev, D, C, L, S, H, dy_dx, gridtype,
                                                 align_corners)
        else:
            with _dfhip.timed("grid_encode_forward", B * (4 * D + L * C * es) + table.numel() * es):
                _backend.grid_encode_forward_blc(inputs, table, offsets, outputs, B, D, C, L, S,
                                                 H, dy_dx, gridtype, align_corners)
        ctx.save_for_backward(inputs, offsets, dy_dx)
        # the live count is read by the backward's kernels at run time (not a
        # saved tensor: the march rewrites its counter row every 16 steps)
        ctx.m_dev = m_dev
        ctx.dims = (B, D, C, L, S, H, gridtype, bool(align_corners), float(bound))
        ctx.table_meta = (table.shape[0], table.dtype, embeddings.dtype)
        ctx.offsets_host = offsets_host
        ctx.backward_mode = backward_mode
        return outputs

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad):
        inputs, offsets, dy_dx = ctx.saved_tensors
        m_dev = ctx.m_dev
        B, D, C, L, S, H, gridtype, align_corners, bound = ctx.dims
        rows, table_dtype, emb_dtype = ctx.table_meta
        nones = (None,) * 10
        grad = grad.to(table_dtype).contiguous()
        if dy_dx is None and ctx.backward_mode == "binned" and binned_eligible(D, C, grad.dtype):
            # [B, L*C] -> the level-major [L, B, C] the walk streams per level
            grad_lbc = torch.empty(L, B, C, dtype=grad.dtype, device=grad.device)
            _backend.grid_grad_blc_to_lbc(grad, grad_lbc, B, L, C)
            offs_h = ctx.offsets_host if ctx.offsets_host is not None else host_offsets(offsets)
            # algorithmic bytes: inputs + grads of the live rows once, the f32
            # table gradient written once
            per = 4 * D + L * C * grad.element_size()
            with _dfhip.timed("grid_encode_backward", 4 * rows * C + (0 if m_dev is not None
                                                                      else B * per),
                              m_dev, per):
                gemb = binned_embedding_grad(grad_lbc, inputs, bound, offsets, offs_h, B, m_dev,
                                             C, L, S, H, gridtype, align_corners)
            return (None, gemb.to(emb_dtype)) + nones
        # the reference's scatter of half2 / f32 atomics (gridencoder.cu:226-313)
        if m_dev is not None:  # the atomic kernels take no device count
            m = int(m_dev[0].item())
            grad, inputs = grad[:m], inputs[:m]
            if dy_dx is not None:
                dy_dx = dy_dx[:m]
            B = m
        x01 = inputs if bound <= 0 else (inputs + bound) / (2 * bound)
        grad_embeddings = torch.zeros(rows, C, device=grad.device, dtype=table_dtype)
        grad_inputs = None
        if dy_dx is not None:
            grad_inputs = torch.empty(B, D, device=grad.device, dtype=table_dtype)
        # HBM algorithmic bytes: grad + inputs per sample (the 2^D*L*C atomic
        # adds per sample are L2/atomic-unit traffic, accounted separately)
        with _dfhip.timed("grid_encode_backward", B * (4 * D + L * C * grad.element_size())):
            _backend.grid_encode_backward_blc(grad, x01.contiguous(), offsets, grad_embeddings, B,
                                              D, C, L, S, H, dy_dx, grad_inputs, gridtype,
                                              align_corners)
        if grad_inputs is not None:
            grad_inputs = grad_inputs.to(inputs.dtype)
            if bound > 0:
                grad_inputs = grad_inputs / (2 * bound)
            if grad_inputs.shape[0] < ctx.dims[0]:  # rows past the live count: no gradient
                full = torch.zeros(ctx.dims[0], D, device=grad.device, dtype=grad_inputs.dtype)
                full[:grad_inputs.shape[0]] = grad_inputs
                grad_inputs = full
        return (grad_inputs, grad_embeddings.to(emb_dtype)) + nones


grid_encode = _grid_encode.apply


def level_offsets(num_levels, level_dim, input_dim, base_resolution, per_level_scale,
                  log2_hashmap_size, align_corners):
    """Row offsets of each level's table (reference grid.py:110-124): rows of
    level l = min(2^log2_hashmap_size, (res_l [+1])^D) rounded up to 8, with
    res_l = ceil(base_resolution * per_level_scale^l)."""
    cap = 2 ** log2_hashmap_size
    starts, total = [], 0
    for lvl in range(num_levels):
        res = int(np.ceil(base_resolution * per_level_scale ** lvl))
        side = res if align_corners else res + 1
        rows = int(np.ceil(min(cap, side ** input_dim) / 8) * 8)
        starts.append(total)
        total += rows
    starts.append(total)
    return np.asarray(starts, dtype=np.int32)


class GridEncoder(nn.Module):
    def __init__(self, input_dim=3, num_levels=16, level_dim=2, per_level_scale=2,
                 base_resolution=16, log2_hashmap_size=19, desired_resolution=None,
                 gridtype="hash", align_corners=False):
        super().__init__()
        if desired_resolution is not None:
            # finest level hits desired_resolution (grid.py:96-97)
            per_level_scale = np.exp2(np.log2(desired_resolution / base_resolution) / (num_levels - 1))
        self.input_dim = input_dim
        self.num_levels = num_levels
        self.level_dim = level_dim
        self.per_level_scale = per_level_scale
        self.log2_hashmap_size = log2_hashmap_size
        self.base_resolution = base_resolution
        self.output_dim = num_levels * level_dim
        self.gridtype = gridtype
        self.gridtype_id = _gridtype_to_id[gridtype]
        self.align_corners = align_corners
        self.max_params = 2 ** log2_hashmap_size
        # embedding backward: "binned" (owner-computes walk, csrc/gridbin.hip)
        # or "atomic" (the reference's scatter, gridencoder.cu:226-313)
        self.backward_mode = "binned"

        offsets = level_offsets(num_levels, level_dim, input_dim, base_resolution,
                                per_level_scale, log2_hashmap_size, align_corners)
        self.register_buffer("offsets", torch.from_numpy(offsets))
        self.offsets_host = offsets  # host copy (the binned backward sizes its slices from it)
        self.n_params = self.offsets[-1] * level_dim
        self.embeddings = nn.Parameter(torch.empty(int(offsets[-1]), level_dim))
        self.reset_parameters()

    def reset_parameters(self):
        std = 1e-4
        self.embeddings.data.uniform_(-std, std)

    def __repr__(self):
        top = int(round(self.base_resolution * self.per_level_scale ** (self.num_levels - 1)))
        return (f"GridEncoder: input_dim={self.input_dim} num_levels={self.num_levels} "
                f"level_dim={self.level_dim} resolution={self.base_resolution} -> {top} "
                f"per_level_scale={self.per_level_scale:.4f} params={tuple(self.embeddings.shape)} "
                f"gridtype={self.gridtype} align_corners={self.align_corners}")

    def forward(self, inputs, bound=1):
        """inputs [..., input_dim] in [-bound, bound] -> [..., num_levels*level_dim].
        Capacity-sized inputs carrying a device live-row count (the
        device-count march) are encoded up to that count; the rest of the rows
        come out as zeros."""
        lead = list(inputs.shape[:-1])
        m_dev = getattr(inputs, _LIVE_ROWS_ATTR, None)
        raw = (inputs.is_cuda and inputs.dtype == torch.float32 and bound > 0
               and not inputs.requires_grad)
        if raw or m_dev is not None:
            # the kernels map (x + bound) / (2 bound) themselves (grid.py:142)
            x = inputs.reshape(-1, self.input_dim)
            if not raw:
                x = ((x + bound) / (2 * bound)).float()
            out = grid_encode(x, self.embeddings, self.offsets, self.per_level_scale,
                              self.base_resolution, x.requires_grad, self.gridtype_id,
                              self.align_corners, self.offsets_host, float(bound) if raw else 0.0,
                              m_dev, self.backward_mode)
        else:
            x = (inputs + bound) / (2 * bound)
            x = x.view(-1, self.input_dim)
            out = grid_encode(x, self.embeddings, self.offsets, self.per_level_scale,
                              self.base_resolution, x.requires_grad, self.gridtype_id,
                              self.align_corners, self.offsets_host, 0.0, None,
                              self.backward_mode)
        out = out.view(lead + [self.output_dim])
        if m_dev is not None:
            # the features of the capacity-sized batch: the same live rows
            setattr(out, _LIVE_ROWS_ATTR, m_dev)
        return out
