"""Python API of the ray-marching ops (mirror of reference raymarching/raymarching.py).

Every public callable keeps the reference's name, argument order, defaults and
return values (raymarching.py:19-373), so `nerf/renderer.py`-style callers run
unchanged.  Differences, all in favour of the GPU and none visible to callers:

* `march_rays_train` is deterministic (rays come back in ray-id order with
  offsets = exclusive prefix sum of the per-ray counts) and never zero-fills
  N*max_steps rows: the emit kernel writes zeros only into the align tail.
  The one host sync of the reference (`step_counter[0].item()`,
  raymarching.py:224) stays, because the returned tensors are sliced to it.
  `torch.cuda.empty_cache()` (raymarching.py:231) is not called: it forces a
  fresh device allocation of the sample buffers every step.
* The backward of `composite_rays_train` writes every row of its gradients
  (no `zeros_like` memset) when the rays come from `march_rays_train`.

There is no CPU path: every op raises if its tensors are not on the GPU.
"""
import torch
from torch.autograd import Function
from torch.amp import custom_bwd, custom_fwd

import _dfhip
import _raymarching as _backend

_fwd_f32 = custom_fwd(device_type="cuda", cast_inputs=torch.float32)
_bwd = custom_bwd(device_type="cuda")

# Set on the `rays` tensor returned by march_rays_train: its rows are in ray-id
# order and their sample ranges tile [0, total) (lets the compositing backward
# write every gradient row itself instead of relying on a memset).
_ORDERED_ATTR = "_dfhip_ray_ordered"


def _flat3(t):
    return t.contiguous().view(-1, 3)


def _to_gpu(t):
    return t if t.is_cuda else t.cuda()


# ----------------------------------------------------------------------------
# utils (raymarching.py:19-155)
# ----------------------------------------------------------------------------

class _near_far_from_aabb(Function):
    @staticmethod
    @_fwd_f32
    def forward(ctx, rays_o, rays_d, aabb, min_near=0.2):
        """Ray / aabb slab intersection.  rays_o, rays_d: [N, 3]; aabb: [6]
        (xmin, ymin, zmin, xmax, ymax, zmax).  Returns nears, fars: [N]; rays
        that miss get FLT_MAX for both."""
        rays_o = _flat3(_to_gpu(rays_o))
        rays_d = _flat3(_to_gpu(rays_d))
        n = rays_o.shape[0]
        nears = torch.empty(n, dtype=rays_o.dtype, device=rays_o.device)
        fars = torch.empty_like(nears)
        _backend.near_far_from_aabb(rays_o, rays_d, _to_gpu(aabb).contiguous(), n, min_near,
                                    nears, fars)
        return nears, fars


near_far_from_aabb = _near_far_from_aabb.apply


class _sph_from_ray(Function):
    @staticmethod
    @_fwd_f32
    def forward(ctx, rays_o, rays_d, radius):
        """(theta, phi) in [-1, 1]^2 where each ray leaves Sphere(radius): [N, 2]."""
        rays_o = _flat3(_to_gpu(rays_o))
        rays_d = _flat3(_to_gpu(rays_d))
        n = rays_o.shape[0]
        coords = torch.empty(n, 2, dtype=rays_o.dtype, device=rays_o.device)
        _backend.sph_from_ray(rays_o, rays_d, radius, n, coords)
        return coords


sph_from_ray = _sph_from_ray.apply


class _morton3D(Function):
    @staticmethod
    def forward(ctx, coords):
        """coords: [N, 3] int32 in [0, 128) -> morton codes [N] int32."""
        coords = _to_gpu(coords).int().contiguous()
        n = coords.shape[0]
        indices = torch.empty(n, dtype=torch.int32, device=coords.device)
        _backend.morton3D(coords, n, indices)
        return indices


morton3D = _morton3D.apply


class _morton3D_invert(Function):
    @staticmethod
    def forward(ctx, indices):
        """indices: [N] int32 -> coords [N, 3] int32."""
        indices = _to_gpu(indices).int().contiguous()
        n = indices.shape[0]
        coords = torch.empty(n, 3, dtype=torch.int32, device=indices.device)
        _backend.morton3D_invert(indices, n, coords)
        return coords


morton3D_invert = _morton3D_invert.apply


class _packbits(Function):
    @staticmethod
    @_fwd_f32
    def forward(ctx, grid, thresh, bitfield=None):
        """grid: [C, H^3] float -> bitfield [C*H^3/8] uint8, bit i of byte n set
        iff grid.flat[8n+i] > thresh.  Written in place into `bitfield` if given."""
        grid = _to_gpu(grid).contiguous()
        n_bytes = grid.shape[0] * grid.shape[1] // 8
        if bitfield is None:
            bitfield = torch.empty(n_bytes, dtype=torch.uint8, device=grid.device)
        _backend.packbits(grid, n_bytes, thresh, bitfield)
        return bitfield


packbits = _packbits.apply


# ----------------------------------------------------------------------------
# training (raymarching.py:161-291)
# ----------------------------------------------------------------------------

def _align_up(m, align):
    # reference rule (raymarching.py:201-202, 225-226): always adds, even when
    # m is already a multiple of align
    return m + align - m % align if align > 0 else m


class _march_rays_train(Function):
    @staticmethod
    @_fwd_f32
    def forward(ctx, rays_o, rays_d, bound, density_bitfield, C, H, nears, fars, step_counter=None,
                mean_count=-1, perturb=False, align=-1, force_all_rays=False, dt_gamma=0,
                max_steps=1024):
        """March rays through the occupancy bitfield and emit occupied samples.

        Returns xyzs [M, 3], dirs [M, 3], deltas [M, 2] (dt, depth delta) and
        rays [N, 3] int32 = (ray id, first sample row, sample count).  With
        force_all_rays (or mean_count <= 0) M is the emitted count rounded up
        by `align`; otherwise M = mean_count rounded up and rays that do not fit
        are dropped (here: the last rays in id order).  `perturb` may also be
        an [N] f32 tensor: the noises to use (replaying another step's draws)."""
        rays_o = _flat3(_to_gpu(rays_o))
        rays_d = _flat3(_to_gpu(rays_d))
        density_bitfield = _to_gpu(density_bitfield).contiguous()
        nears = nears.contiguous()
        fars = fars.contiguous()
        n = rays_o.shape[0]
        dev, dt = rays_o.device, rays_o.dtype

        if step_counter is None:
            step_counter = torch.zeros(2, dtype=torch.int32, device=dev)
        if torch.is_tensor(perturb):
            noises = perturb.to(dt).contiguous()
        else:
            noises = (torch.rand(n, dtype=dt, device=dev) if perturb
                      else torch.zeros(n, dtype=dt, device=dev))
        rays = torch.empty(n, 3, dtype=torch.int32, device=dev)
        block_sums = torch.empty(_backend.march_rays_train_scratch_ints(n), dtype=torch.int32,
                                 device=dev)

        exact = force_all_rays or mean_count <= 0
        if exact:
            cap = n * max_steps
            zero_tail = align if align > 0 else 0  # nothing past m is returned
        else:
            cap = _align_up(mean_count, align)
            zero_tail = -1
        # rows are written by the emit pass (and its tail zeroing) only
        xyzs = torch.empty(cap, 3, dtype=dt, device=dev)
        dirs = torch.empty(cap, 3, dtype=dt, device=dev)
        deltas = torch.empty(cap, 2, dtype=dt, device=dev)

        # per ray: o, d, near, far, noise in; (id, offset, count) out; bitfield once
        ray_bytes = n * (4 * 9 + 12) + density_bitfield.numel()
        # exact form: the count pass keeps every sample in a stage buffer and
        # the emit only copies it into ray order (no second march)
        stage = (torch.empty(_backend.march_rays_train_stage_floats(n, max_steps), dtype=dt,
                             device=dev) if exact and dt == torch.float32 else None)
        with _dfhip.timed("march_rays_train_count", ray_bytes):
            if stage is not None:
                _backend.march_rays_train_count_staged(rays_o, rays_d, density_bitfield, bound,
                                                       dt_gamma, max_steps, n, C, H, nears, fars,
                                                       rays, step_counter, noises, block_sums,
                                                       stage)
            else:
                _backend.march_rays_train_count(rays_o, rays_d, density_bitfield, bound,
                                                dt_gamma, max_steps, n, C, H, nears, fars, rays,
                                                step_counter, noises, block_sums)
        emit_region = _dfhip.timed("march_rays_train_emit", ray_bytes)
        with emit_region:  # + 32 B per written sample, added below once known
            if stage is not None:
                _backend.march_rays_train_emit_staged(rays_d, max_steps, n, cap, xyzs, dirs,
                                                      deltas, rays, block_sums, zero_tail, stage)
            else:
                _backend.march_rays_train_emit(rays_o, rays_d, density_bitfield, bound, dt_gamma,
                                               max_steps, n, C, H, cap, nears, fars, xyzs, dirs,
                                               deltas, rays, noises, block_sums, zero_tail)
        if exact:
            m = _align_up(int(step_counter[0].item()), align)  # D2H sync (as the reference)
            xyzs, dirs, deltas = xyzs[:m], dirs[:m], deltas[:m]
        if emit_region is not _dfhip._NO_REGION:
            emit_region.nbytes += 32 * xyzs.shape[0]
        setattr(rays, _ORDERED_ATTR, True)
        ctx.mark_non_differentiable(xyzs, dirs, deltas, rays)
        return xyzs, dirs, deltas, rays


march_rays_train = _march_rays_train.apply

# Set on the capacity-sized tensors returned by march_rays_train_dev: an int32
# device view of the live sample count (consumers that honour it, the fused
# grid field and the mixed compositing, stop there; anything else reads the
# whole capacity, which is correct but slower).
LIVE_ROWS_ATTR = "_dfhip_live_rows"


def live_rows(t):
    """The int32 device view of the live row count attached to `t`, or None."""
    return getattr(t, LIVE_ROWS_ATTR, None)


@torch.no_grad()
def march_rays_train_dev(rays_o, rays_d, bound, density_bitfield, C, H, nears, fars, step_counter,
                         perturb=False, dt_gamma=0, max_steps=1024, noises=None):
    """Native form of march_rays_train(..., force_all_rays=True) with NO host
    synchronisation (so a whole train step can be captured in a HIP graph).

    Same samples, in the same ray order, as march_rays_train; the difference is
    the shape: xyzs / dirs / deltas come back at their capacity N * max_steps
    rows (only rows [0, step_counter[0]) are written) instead of being sliced
    to the align-rounded count, which needs the count on the host
    (reference raymarching.py:224).  Each returned tensor carries
    `live_rows(t)` = step_counter[0:1]."""
    rays_o = _flat3(rays_o)
    rays_d = _flat3(rays_d)
    n = rays_o.shape[0]
    dev = rays_o.device
    rays_o = rays_o.float()
    rays_d = rays_d.float()
    nears = nears.float().contiguous()
    fars = fars.float().contiguous()
    if noises is None:  # (given: the draws of another step, tests/test_gpu_native_step.py)
        noises = (torch.rand(n, device=dev) if perturb else torch.zeros(n, device=dev))
    rays = torch.empty(n, 3, dtype=torch.int32, device=dev)
    block_sums = torch.empty(_backend.march_rays_train_scratch_ints(n), dtype=torch.int32,
                             device=dev)
    cap = n * max_steps
    xyzs = torch.empty(cap, 3, device=dev)
    dirs = torch.empty(cap, 3, device=dev)
    deltas = torch.empty(cap, 2, device=dev)
    density_bitfield = density_bitfield.contiguous()
    ray_bytes = n * (4 * 9 + 12) + density_bitfield.numel()
    with _dfhip.timed("march_rays_train_count", ray_bytes):
        _backend.march_rays_train_count(rays_o, rays_d, density_bitfield, bound, dt_gamma,
                                        max_steps, n, C, H, nears, fars, rays, step_counter,
                                        noises, block_sums)
    m_dev = step_counter[:1]
    with _dfhip.timed("march_rays_train_emit", ray_bytes, m_dev, 32):
        _backend.march_rays_train_emit(rays_o, rays_d, density_bitfield, bound, dt_gamma,
                                       max_steps, n, C, H, cap, nears, fars, xyzs, dirs, deltas,
                                       rays, noises, block_sums, 0)
    for t in (xyzs, dirs, deltas, rays):
        setattr(t, LIVE_ROWS_ATTR, m_dev)
    setattr(rays, _ORDERED_ATTR, True)
    return xyzs, dirs, deltas, rays


class _composite_rays_train(Function):
    @staticmethod
    @custom_fwd(device_type="cuda")
    def forward(ctx, sigmas, rgbs, deltas, rays, T_thresh=1e-4):
        """Front-to-back alpha compositing of each ray's samples.

        sigmas [M], rgbs [M, 3], deltas [M, 2], rays [N, 3] -> weights_sum [N],
        depth [N], image [N, 3] (colour already multiplied by alpha).

        Under autocast every input is cast to float32 as the reference's
        custom_fwd(cast_inputs=torch.float32) does, except that f16 colours of
        ray-ordered samples are read (and their gradient written) as f16 by the
        mixed kernels: the f16 -> f32 cast is exact and the reference's
        autograd rounds the f32 colour gradient to f16 once, so the numbers are
        the same without the two [M, 3] cast passes.  bf16 colours (bf16
        autocast, the C5 option) take the same route."""
        ordered = bool(getattr(rays, _ORDERED_ATTR, False))
        if torch.is_autocast_enabled("cuda"):
            sigmas, deltas = sigmas.float(), deltas.float()
            if not (ordered and rgbs.dtype in (torch.float16, torch.bfloat16)):
                rgbs = rgbs.float()
        sigmas = sigmas.contiguous()
        rgbs = rgbs.contiguous()
        deltas = deltas.contiguous()
        m, n = sigmas.shape[0], rays.shape[0]
        # f32 sigmas with f16/f32 colours of ray-ordered samples: mixed kernels
        mixed = (ordered and sigmas.dtype == torch.float32 and deltas.dtype == torch.float32
                 and rgbs.dtype in (torch.float16, torch.bfloat16, torch.float32))
        opts = dict(dtype=sigmas.dtype, device=sigmas.device)
        weights_sum = torch.empty(n, **opts)
        depth = torch.empty(n, **opts)
        image = torch.empty(n, 3, **opts)
        live = live_rows(rays)
        with _dfhip.timed("composite_rays_train_forward", 32 * n + (24 * m if live is None else 0),
                          live, 24):
            fn = (_backend.composite_rays_train_forward_mixed if mixed
                  else _backend.composite_rays_train_forward)
            fn(sigmas, rgbs, deltas, rays, m, n, T_thresh, weights_sum, depth, image)
        ctx.save_for_backward(sigmas, rgbs, deltas, rays, weights_sum, depth, image)
        ctx.dims = (m, n, T_thresh)
        ctx.ordered = ordered
        ctx.mixed = mixed
        # capacity-sized samples (march_rays_train_dev): rows past the live
        # count are never read downstream, so the backward need not zero them
        ctx.live = live
        ctx.zero_tail = live is None
        return weights_sum, depth, image

    @staticmethod
    @_bwd
    def backward(ctx, grad_weights_sum, grad_depth, grad_image):
        # grad_depth is not propagated (reference raymarching.py:275)
        sigmas, rgbs, deltas, rays, weights_sum, depth, image = ctx.saved_tensors
        m, n, T_thresh = ctx.dims
        grad_weights_sum = grad_weights_sum.contiguous()
        grad_image = grad_image.contiguous()
        nbytes = 40 * m + 44 * n
        if ctx.mixed:
            grad_sigmas = torch.empty_like(sigmas)
            grad_rgbs = torch.empty_like(rgbs)
            live = ctx.live
            with _dfhip.timed("composite_rays_train_backward",
                              nbytes if live is None else 44 * n, live, 40):
                _backend.composite_rays_train_backward_mixed(
                    grad_weights_sum.float(), grad_image.float(), sigmas, rgbs, deltas, rays,
                    weights_sum, image, m, n, T_thresh, grad_sigmas, grad_rgbs, ctx.zero_tail)
            return grad_sigmas, grad_rgbs, None, None, None
        if ctx.ordered:
            grad_sigmas = torch.empty_like(sigmas)
            grad_rgbs = torch.empty_like(rgbs)
            fn = _backend.composite_rays_train_backward_dense
        else:
            grad_sigmas = torch.zeros_like(sigmas)
            grad_rgbs = torch.zeros_like(rgbs)
            fn = _backend.composite_rays_train_backward
        with _dfhip.timed("composite_rays_train_backward", nbytes):
            fn(grad_weights_sum, grad_image, sigmas, rgbs, deltas, rays, weights_sum, image, m, n,
               T_thresh, grad_sigmas, grad_rgbs)
        return grad_sigmas, grad_rgbs, None, None, None


composite_rays_train = _composite_rays_train.apply


# ----------------------------------------------------------------------------
# inference (raymarching.py:297-373)
# ----------------------------------------------------------------------------

class _march_rays(Function):
    @staticmethod
    @_fwd_f32
    def forward(ctx, n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, density_bitfield,
                C, H, near, far, align=-1, perturb=False, dt_gamma=0, max_steps=1024):
        """Advance each alive ray by up to n_step occupied samples from rays_t.
        Returns xyzs/dirs [n_alive*n_step (+align pad), 3], deltas [.., 2];
        unused slots are zero (a zero delta marks the end of a ray)."""
        rays_o = _flat3(_to_gpu(rays_o))
        rays_d = _flat3(_to_gpu(rays_d))
        dev, dt = rays_o.device, rays_o.dtype
        rows = n_alive * n_step
        m = rows + (align - rows % align) if align > 0 else rows
        xyzs = torch.empty(m, 3, dtype=dt, device=dev)
        dirs = torch.empty(m, 3, dtype=dt, device=dev)
        deltas = torch.empty(m, 2, dtype=dt, device=dev)
        if m > rows:  # the kernel fills every slot of the alive rays
            xyzs[rows:].zero_()
            dirs[rows:].zero_()
            deltas[rows:].zero_()
        noises = (torch.rand(n_alive, dtype=dt, device=dev) if perturb
                  else torch.zeros(n_alive, dtype=dt, device=dev))
        _backend.march_rays(n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, dt_gamma,
                            max_steps, C, H, density_bitfield.contiguous(), near, far, xyzs, dirs,
                            deltas, noises)
        return xyzs, dirs, deltas


march_rays = _march_rays.apply


class _composite_rays(Function):
    @staticmethod
    @_fwd_f32
    def forward(ctx, n_alive, n_step, rays_alive, rays_t, sigmas, rgbs, deltas, weights_sum, depth,
                image, T_thresh=1e-2):
        """In-place compositing step of the inference loop: accumulates into
        weights_sum / depth / image, marks terminated rays with rays_alive = -1
        and advances rays_t of the others."""
        _backend.composite_rays(n_alive, n_step, T_thresh, rays_alive, rays_t,
                                sigmas.contiguous(), rgbs.contiguous(), deltas.contiguous(),
                                weights_sum, depth, image)
        return tuple()


composite_rays = _composite_rays.apply
