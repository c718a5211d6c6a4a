"""`_raymarching` backend module: the reference pybind11 surface
(raymarching/src/bindings.cpp:5-18) over the gfx950 C-ABI (include/dfhip.h).

Same argument order and in-place output convention as the reference: the
caller allocates every output, the function returns None.  Unlike the
reference (no checks, raymarching.cu:13-16 unused), device / contiguity /
dtype are validated and raise RuntimeError.
"""
import torch

import _dfhip as _d
from _dfhip import call, ptr, stream, checked


def _f(t, what):
    checked(t, what)
    return _d.dtype_code(t, what)


def packbits(grid, N, density_thresh, bitfield):
    dt = _f(grid, "grid")
    checked(bitfield, "bitfield", "u8")
    call("dfhip_packbits", dt, ptr(grid), N, density_thresh, ptr(bitfield), stream())


def near_far_from_aabb(rays_o, rays_d, aabb, N, min_near, nears, fars):
    dt = _f(rays_o, "rays_o")
    for t, w in ((rays_d, "rays_d"), (aabb, "aabb"), (nears, "nears"), (fars, "fars")):
        checked(t, w)
    call("dfhip_near_far_from_aabb", dt, ptr(rays_o), ptr(rays_d), ptr(aabb), N, min_near,
         ptr(nears), ptr(fars), stream())


def sph_from_ray(rays_o, rays_d, radius, N, coords):
    dt = _f(rays_o, "rays_o")
    checked(rays_d, "rays_d")
    checked(coords, "coords")
    call("dfhip_sph_from_ray", dt, ptr(rays_o), ptr(rays_d), radius, N, ptr(coords), stream())


def morton3D(coords, N, indices):
    checked(coords, "coords", "int")
    checked(indices, "indices", "int")
    call("dfhip_morton3D", ptr(coords), N, ptr(indices), stream())


def morton3D_invert(indices, N, coords):
    checked(indices, "indices", "int")
    checked(coords, "coords", "int")
    call("dfhip_morton3D_invert", ptr(indices), N, ptr(coords), stream())


def march_rays_train(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, M, nears, fars,
                     xyzs, dirs, deltas, rays, counter, noises):
    dt = _f(rays_o, "rays_o")
    checked(grid, "grid", "u8")
    checked(rays, "rays", "int")
    checked(counter, "counter", "int")
    call("dfhip_march_rays_train", dt, ptr(rays_o), ptr(rays_d), ptr(grid), bound, dt_gamma,
         max_steps, N, C, H, M, ptr(nears), ptr(fars), ptr(xyzs), ptr(dirs), ptr(deltas),
         ptr(rays), ptr(counter), ptr(noises), stream())


# ---- native split form (deterministic count / emit; see dfhip.h)

def march_rays_train_scratch_ints(N):
    return int(_d.load().dfhip_march_rays_train_scratch_ints(N))


def march_rays_train_count(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, nears, fars,
                           rays, counter, noises, block_sums):
    dt = _f(rays_o, "rays_o")
    checked(grid, "grid", "u8")
    checked(block_sums, "block_sums", "int")
    call("dfhip_march_rays_train_count", dt, ptr(rays_o), ptr(rays_d), ptr(grid), bound, dt_gamma,
         max_steps, N, C, H, ptr(nears), ptr(fars), ptr(rays), ptr(counter), ptr(noises),
         ptr(block_sums), stream())


def march_rays_train_emit(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, M, nears,
                          fars, xyzs, dirs, deltas, rays, noises, block_sums, zero_tail):
    dt = _f(rays_o, "rays_o")
    call("dfhip_march_rays_train_emit", dt, ptr(rays_o), ptr(rays_d), ptr(grid), bound, dt_gamma,
         max_steps, N, C, H, M, ptr(nears), ptr(fars), ptr(xyzs), ptr(dirs), ptr(deltas),
         ptr(rays), ptr(noises), ptr(block_sums), int(zero_tail), stream())


def march_rays_train_stage_floats(N, max_steps):
    return int(_d.load().dfhip_march_rays_train_stage_floats(int(N), int(max_steps)))


def march_rays_train_count_staged(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, nears,
                                  fars, rays, counter, noises, block_sums, stage):
    """march_rays_train_count that also keeps every sample in `stage` (f32,
    march_rays_train_stage_floats(N, max_steps) floats)."""
    dt = _f(rays_o, "rays_o")
    checked(grid, "grid", "u8")
    checked(block_sums, "block_sums", "int")
    checked(stage, "stage")
    if stage.dtype != torch.float32 or stage.numel() < march_rays_train_stage_floats(N, max_steps):
        raise RuntimeError("stage must be float32 with march_rays_train_stage_floats(N, max_steps) "
                           "elements")
    call("dfhip_march_rays_train_count_staged", dt, ptr(rays_o), ptr(rays_d), ptr(grid), bound,
         dt_gamma, max_steps, N, C, H, ptr(nears), ptr(fars), ptr(rays), ptr(counter),
         ptr(noises), ptr(block_sums), ptr(stage), stream())


def march_rays_train_emit_staged(rays_d, max_steps, N, M, xyzs, dirs, deltas, rays, block_sums,
                                 zero_tail, stage):
    """march_rays_train_emit from the count pass's stage (no second march)."""
    dt = _f(rays_d, "rays_d")
    checked(stage, "stage")
    call("dfhip_march_rays_train_emit_staged", dt, ptr(rays_d), max_steps, N, M, ptr(xyzs),
         ptr(dirs), ptr(deltas), ptr(rays), ptr(block_sums), int(zero_tail), ptr(stage), stream())


def composite_rays_train_forward(sigmas, rgbs, deltas, rays, M, N, T_thresh, weights_sum, depth,
                                 image):
    dt = _f(sigmas, "sigmas")
    for t, w in ((rgbs, "rgbs"), (deltas, "deltas"), (weights_sum, "weights_sum"),
                 (depth, "depth"), (image, "image")):
        checked(t, w)
    checked(rays, "rays", "int")
    call("dfhip_composite_rays_train_forward", dt, ptr(sigmas), ptr(rgbs), ptr(deltas), ptr(rays),
         M, N, T_thresh, ptr(weights_sum), ptr(depth), ptr(image), stream())


def _composite_bwd(name, grad_weights_sum, grad_image, sigmas, rgbs, deltas, rays, weights_sum,
                   image, M, N, T_thresh, grad_sigmas, grad_rgbs):
    dt = _f(grad_image, "grad_image")
    for t, w in ((grad_weights_sum, "grad_weights_sum"), (sigmas, "sigmas"), (rgbs, "rgbs"),
                 (deltas, "deltas"), (weights_sum, "weights_sum"), (image, "image"),
                 (grad_sigmas, "grad_sigmas"), (grad_rgbs, "grad_rgbs")):
        checked(t, w)
    call(name, dt, ptr(grad_weights_sum), ptr(grad_image), ptr(sigmas), ptr(rgbs), ptr(deltas),
         ptr(rays), ptr(weights_sum), ptr(image), M, N, T_thresh, ptr(grad_sigmas),
         ptr(grad_rgbs), stream())


def composite_rays_train_backward(*args):
    _composite_bwd("dfhip_composite_rays_train_backward", *args)


def composite_rays_train_backward_dense(*args):
    _composite_bwd("dfhip_composite_rays_train_backward_dense", *args)


# ---- native mixed-precision train compositing (f32 sigmas, f16/f32 colours)

def _f32_only(t, what):
    checked(t, what)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{what} must be a float32 tensor")


def composite_rays_train_forward_mixed(sigmas, rgbs, deltas, rays, M, N, T_thresh, weights_sum,
                                       depth, image):
    for t, w in ((sigmas, "sigmas"), (deltas, "deltas"), (weights_sum, "weights_sum"),
                 (depth, "depth"), (image, "image")):
        _f32_only(t, w)
    rd = _f(rgbs, "rgbs")
    checked(rays, "rays", "int")
    call("dfhip_composite_rays_train_forward_mixed", rd, ptr(sigmas), ptr(rgbs), ptr(deltas),
         ptr(rays), M, N, T_thresh, ptr(weights_sum), ptr(depth), ptr(image), stream())


def composite_rays_train_backward_mixed(grad_weights_sum, grad_image, sigmas, rgbs, deltas, rays,
                                        weights_sum, image, M, N, T_thresh, grad_sigmas,
                                        grad_rgbs, zero_tail=True):
    for t, w in ((grad_weights_sum, "grad_weights_sum"), (grad_image, "grad_image"),
                 (sigmas, "sigmas"), (deltas, "deltas"), (weights_sum, "weights_sum"),
                 (image, "image"), (grad_sigmas, "grad_sigmas")):
        _f32_only(t, w)
    rd = _f(rgbs, "rgbs")
    checked(grad_rgbs, "grad_rgbs")
    if grad_rgbs.dtype != rgbs.dtype:
        raise RuntimeError("grad_rgbs must have the dtype of rgbs")
    checked(rays, "rays", "int")
    call("dfhip_composite_rays_train_backward_mixed", rd, ptr(grad_weights_sum), ptr(grad_image),
         ptr(sigmas), ptr(rgbs), ptr(deltas), ptr(rays), ptr(weights_sum), ptr(image), M, N,
         T_thresh, ptr(grad_sigmas), ptr(grad_rgbs), int(bool(zero_tail)), stream())


def march_rays(n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, bound, dt_gamma, max_steps, C,
               H, grid, near, far, xyzs, dirs, deltas, noises):
    dt = _f(rays_o, "rays_o")
    checked(rays_alive, "rays_alive", "int")
    checked(grid, "grid", "u8")
    call("dfhip_march_rays", dt, n_alive, n_step, ptr(rays_alive), ptr(rays_t), ptr(rays_o),
         ptr(rays_d), bound, dt_gamma, max_steps, C, H, ptr(grid), ptr(near), ptr(far), ptr(xyzs),
         ptr(dirs), ptr(deltas), ptr(noises), stream())


def composite_rays(n_alive, n_step, T_thresh, rays_alive, rays_t, sigmas, rgbs, deltas, weights,
                   depth, image):
    dt = _f(image, "image")
    checked(rays_alive, "rays_alive", "int")
    for t, w in ((rays_t, "rays_t"), (sigmas, "sigmas"), (rgbs, "rgbs"), (deltas, "deltas"),
                 (weights, "weights"), (depth, "depth")):
        checked(t, w)
    call("dfhip_composite_rays", dt, n_alive, n_step, T_thresh, ptr(rays_alive), ptr(rays_t),
         ptr(sigmas), ptr(rgbs), ptr(deltas), ptr(weights), ptr(depth), ptr(image), stream())
