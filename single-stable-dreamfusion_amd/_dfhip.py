"""ctypes binding of the gfx950 kernel library (lib/libdfhip.so, include/dfhip.h).

This is the only place that touches the C-ABI.  The per-extension shim modules
(`_raymarching`, `_gridencoder`, `_freqencoder`, `_shencoder`) sit on top of it
and expose the reference's pybind11 signatures.

There is deliberately no CPU / eager fallback: if the library is missing, or a
tensor is not on the GPU, calls raise.  `import torch` happens before the
library is opened, so its HIP runtime dependency (SONAME libamdhip64.so.7)
binds to the runtime torch already loaded and pointers / streams are shared.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

LIB_PATH = Path(os.environ.get("DFHIP_LIB", Path(__file__).resolve().parent / "lib" / "libdfhip.so"))

F32, F16, F64, BF16 = 0, 1, 2, 3
_DTYPE = {torch.float32: F32, torch.float16: F16, torch.float64: F64, torch.bfloat16: BF16}

_vp, _u32, _i32, _f32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_float
_u64 = ctypes.c_uint64

# name -> argtypes (stream is always the trailing c_void_p)
_SIGS = {
    "dfhip_near_far_from_aabb": [_i32, _vp, _vp, _vp, _u32, _f32, _vp, _vp, _vp],
    "dfhip_get_rays": [_vp, _f32, _f32, _f32, _f32, _u32, _u32, _vp, _vp, _vp],
    "dfhip_density_grid_ema": [_vp, _vp, _u32, _u32, _f32, _vp, _vp, _vp],
    "dfhip_packbits_mean": [_vp, _u32, _vp, _f32, _vp, _vp, _vp],
    "dfhip_mean_count": [_vp, _u32, _vp, _vp],
    "dfhip_sph_from_ray": [_i32, _vp, _vp, _f32, _u32, _vp, _vp],
    "dfhip_morton3D": [_vp, _u32, _vp, _vp],
    "dfhip_morton3D_invert": [_vp, _u32, _vp, _vp],
    "dfhip_packbits": [_i32, _vp, _u32, _f32, _vp, _vp],
    "dfhip_march_rays_train": [_i32, _vp, _vp, _vp, _f32, _f32, _u32, _u32, _u32, _u32, _u32,
                               _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_march_rays_train_count": [_i32, _vp, _vp, _vp, _f32, _f32, _u32, _u32, _u32, _u32,
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_march_rays_train_emit": [_i32, _vp, _vp, _vp, _f32, _f32, _u32, _u32, _u32, _u32,
                                    _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "dfhip_march_rays_train_count_staged": [_i32, _vp, _vp, _vp, _f32, _f32, _u32, _u32, _u32,
                                            _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_march_rays_train_emit_staged": [_i32, _vp, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _vp,
                                           _i32, _vp, _vp],
    "dfhip_composite_rays_train_forward": [_i32, _vp, _vp, _vp, _vp, _u32, _u32, _f32, _vp, _vp,
                                           _vp, _vp],
    "dfhip_composite_rays_train_backward": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32,
                                            _u32, _f32, _vp, _vp, _vp],
    "dfhip_composite_rays_train_backward_dense": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                  _u32, _u32, _f32, _vp, _vp, _vp],
    "dfhip_composite_rays_train_forward_mixed": [_i32, _vp, _vp, _vp, _vp, _u32, _u32, _f32,
                                                 _vp, _vp, _vp, _vp],
    "dfhip_composite_rays_train_backward_mixed": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                  _u32, _u32, _f32, _vp, _vp, _i32, _vp],
    "dfhip_march_rays": [_i32, _u32, _u32, _vp, _vp, _vp, _vp, _f32, _f32, _u32, _u32, _u32, _vp,
                         _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_composite_rays": [_i32, _u32, _u32, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_grid_encode_forward": [_i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _f32, _u32,
                                  _vp, _u32, _i32, _vp],
    "dfhip_grid_encode_forward_blc": [_i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _f32,
                                      _u32, _vp, _u32, _i32, _vp],
    "dfhip_grid_encode_forward_dyn": [_i32, _vp, _f32, _vp, _vp, _vp, _u32, _vp, _u32, _u32,
                                      _u32, _f32, _u32, _vp, _u32, _i32, _vp],
    "dfhip_grid_encode_backward": [_i32, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _f32,
                                   _u32, _vp, _vp, _u32, _i32, _vp],
    "dfhip_grid_encode_backward_blc": [_i32, _i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32,
                                       _f32, _u32, _vp, _vp, _u32, _i32, _vp],
    "dfhip_grid_encode_backward_sliced": [_i32, _i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32,
                                          _u32, _f32, _u32, _u32, _i32, _vp, _u32, _i32, _vp],
    "dfhip_grid_encode_backward_sliced_dyn": [_i32, _i32, _vp, _vp, _f32, _vp, _vp, _u32, _u32,
                                              _vp, _u32, _u32, _u32, _f32, _u32, _u32, _i32, _vp,
                                              _u32, _i32, _vp],
    "dfhip_grid_backward_binned_scratch": [_u32, _vp, _u32, _u32, _vp, _vp, _vp],
    "dfhip_grid_encode_backward_binned": [_i32, _vp, _vp, _f32, _vp, _vp, _vp, _u32, _vp, _u32,
                                          _u32, _u32, _f32, _u32, _u32, _i32, _vp, _vp, _vp,
                                          _i32, _vp],
    "dfhip_grid_encode_backward_binned_phase": [_i32, _i32, _vp, _vp, _f32, _vp, _vp, _vp, _u32,
                                                _vp, _u32, _u32, _u32, _f32, _u32, _u32, _i32,
                                                _vp, _vp, _vp, _i32, _vp],
    "dfhip_grid_encode_backward_binned_stencil": [_i32, _i32, _vp, _vp, _f32, _vp, _vp, _vp,
                                                  _u32, _vp, _u32, _u32, _u32, _f32, _u32, _u32,
                                                  _i32, _u32, _f32, _vp, _vp, _vp, _i32, _vp],
    "dfhip_grid_backward_binned_scratch_opts": [_u32, _vp, _u32, _u32, _u32, _vp, _vp, _vp,
                                                _vp],
    "dfhip_grid_encode_backward_binned_opts": [_i32, _i32, _vp, _vp, _f32, _vp, _vp, _vp, _u32,
                                               _vp, _u32, _u32, _u32, _f32, _u32, _u32, _i32,
                                               _u32, _f32, _vp, _vp, _vp, _i32, _vp, _vp],
    "dfhip_grid_grad_blc_to_lbc": [_i32, _vp, _vp, _u32, _u32, _u32, _vp],
    "dfhip_field_mlp_forward": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _u32, _vp],
    "dfhip_field_mlp_backward": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _u32, _vp,
                                 _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "dfhip_mlp_forward": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp],
    "dfhip_mlp_backward": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp,
                           _u32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "dfhip_grid_field_forward": [_vp, _f32, _vp, _vp, _u32, _f32, _u32, _u32, _i32, _vp, _vp, _vp,
                                 _vp, _vp, _vp, _vp, _vp, _vp, _i32, _u32, _vp, _vp],
    "dfhip_grid_field_backward": [_vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32,
                                  _u32, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _u32, _u32, _f32, _u32, _u32, _i32, _vp, _vp, _u32, _vp],
    "dfhip_shading_stencil": [_vp, _vp, _u32, _f32, _f32, _vp, _vp, _vp],
    "dfhip_shading_forward": [_vp, _vp, _vp, _vp, _f32, _f32, _i32, _vp, _u32, _vp, _vp, _vp,
                              _vp, _f32, _vp, _vp, _vp],
    "dfhip_shading_backward": [_vp, _vp, _vp, _vp, _f32, _f32, _i32, _vp, _u32, _vp, _vp, _vp,
                               _f32, _vp, _vp, _vp],
    "dfhip_shading_forward_bf16": [_vp, _vp, _vp, _vp, _f32, _f32, _i32, _vp, _u32, _vp, _vp,
                                   _vp, _vp, _f32, _vp, _vp, _vp],
    "dfhip_shading_backward_bf16": [_vp, _vp, _vp, _vp, _f32, _f32, _i32, _vp, _u32, _vp, _vp,
                                    _vp, _f32, _vp, _vp, _vp],
    "dfhip_shading_light": [_vp, _u64, _u64, _vp, _vp],
    "dfhip_grid_quads": [_i32, _vp, _vp, _u32, _f32, _u32, _u32, _i32, _u32, _vp, _vp, _vp],
    "dfhip_grid_field_forward_quads": [_i32, _vp, _f32, _vp, _vp, _vp, _u32, _f32, _u32, _u32,
                                       _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32,
                                       _u32, _vp, _vp],
    "dfhip_grid_field_forward_bf16": [_vp, _f32, _vp, _vp, _u32, _f32, _u32, _u32, _i32, _vp,
                                      _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _u32, _vp,
                                      _vp],
    "dfhip_grid_field_backward_bf16": [_vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _i32, _u32, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _i32, _vp],
    "dfhip_grid_field_backward_accumulate": [
        _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _u32, _vp, _vp, _vp, _u32,
        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _f32, _u32, _u32, _i32, _vp, _vp, _u32,
        _vp],
    "dfhip_adam_amp_step": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                            _vp, _vp, _f32, _f32, _i32, _vp],
    "dfhip_adam_amp_step_lr_dev": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _f32, _f32, _i32, _vp],
    "dfhip_ray_head_forward": [_u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp],
    "dfhip_ray_head_backward": [_u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                _vp, _vp, _vp, _vp, _vp],
    "dfhip_ray_head_backward_entropy": [_u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp],
    "dfhip_ray_head_forward_backward_entropy_loss": [_u32] + [_vp] * 22 + [_f32, _vp, _vp],
    "dfhip_ray_head_backward_entropy_loss": [_u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                             _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp,
                                             _vp],
    "dfhip_entropy_forward": [_u32, _vp, _f32, _vp, _vp],
    "dfhip_entropy_backward": [_u32, _vp, _vp, _f32, _vp, _vp],
    "dfhip_entropy_backward_accumulate": [_u32, _vp, _vp, _f32, _vp, _vp],
    "dfhip_train_step_prologue": [_vp, _f32, _f32, _f32, _f32, _u32, _u32, _vp, _f32,
                                  ctypes.c_uint64, ctypes.c_uint64, _i32, _vp, _u32, _u32, _vp,
                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_train_step_prologue_lr": [_vp, _f32, _f32, _f32, _f32, _u32, _u32, _vp, _f32,
                                     ctypes.c_uint64, ctypes.c_uint64, _i32, _vp, _u32, _u32,
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp,
                                     _vp],
    "dfhip_render_rays_infer": [_u32, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _u32, _u32, _u32, _vp,
                                _f32, _vp, _vp, _u32, _f32, _u32, _u32, _i32, _vp, _vp, _vp, _vp,
                                _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_render_rays_infer_prof": [_u32, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _u32, _u32, _u32,
                                     _vp, _f32, _vp, _vp, _u32, _f32, _u32, _u32, _i32, _vp, _vp,
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dfhip_render_rays_infer_ordered": [_u32, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _u32, _u32,
                                        _u32, _vp, _f32, _vp, _vp, _u32, _f32, _u32, _u32, _i32,
                                        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                        _u32, _u32, _vp, _vp],
    "dfhip_render_ray_order": [_vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp],
    "dfhip_render_ray_order_occ": [_vp, _vp, _vp, _vp, _vp, _f32, _u32, _u32, _u32, _u32, _u32,
                                   _u32, _vp, _vp, _vp],
    "dfhip_freq_encode_forward": [_vp, _u32, _u32, _u32, _u32, _vp, _vp],
    "dfhip_freq_encode_backward": [_vp, _vp, _u32, _u32, _u32, _u32, _vp, _vp],
    "dfhip_sh_encode_forward": [_i32, _vp, _vp, _u32, _u32, _u32, _vp, _vp],
    "dfhip_sh_encode_backward": [_i32, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp],
}

_lib = None


def load() -> ctypes.CDLL:
    """Open libdfhip.so once and declare every entry point's signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(
            f"gfx950 kernel library not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = ctypes.CDLL(str(LIB_PATH))
    lib.dfhip_last_error.restype = ctypes.c_char_p
    lib.dfhip_abi_version.restype = ctypes.c_int
    # the library must be built from the header these signatures follow: a
    # stale one would be called with other argument lists (and crash)
    from dfhip_build import HEADER, abi_hash
    if not HEADER.exists():
        raise ImportError(f"{HEADER} not found: cannot check the ABI of {LIB_PATH}")
    want, got = abi_hash(HEADER), int(lib.dfhip_abi_version())
    if got != want:
        raise ImportError(
            f"{LIB_PATH} was built from another include/dfhip.h (ABI {got:#x}, header "
            f"{want:#x}); rebuild it: python -c 'import __graft_entry__ as g; g.build()'")
    lib.dfhip_march_rays_train_scratch_ints.restype = _u32
    lib.dfhip_march_rays_train_scratch_ints.argtypes = [_u32]
    lib.dfhip_grid_backward_default_parts.restype = _u32
    lib.dfhip_grid_backward_default_parts.argtypes = [_u32, _u32]
    lib.dfhip_field_mlp_params.restype = _u32
    lib.dfhip_field_mlp_params.argtypes = []
    lib.dfhip_field_mlp_backward_parts.restype = _u32
    lib.dfhip_field_mlp_backward_parts.argtypes = [_u32]
    lib.dfhip_ray_head_partial_floats.restype = _u32
    lib.dfhip_ray_head_partial_floats.argtypes = [_u32]
    lib.dfhip_grid_backward_partial_floats.restype = ctypes.c_uint64
    lib.dfhip_grid_backward_partial_floats.argtypes = [_u32, _u32, _u32]
    lib.dfhip_shading_partial_doubles.restype = _u32
    lib.dfhip_shading_partial_doubles.argtypes = [_u32]
    lib.dfhip_grid_backward_binned_tile.restype = _u32
    lib.dfhip_grid_backward_binned_tile.argtypes = [_u32, _vp]
    lib.dfhip_march_rays_train_stage_floats.restype = ctypes.c_uint64
    lib.dfhip_march_rays_train_stage_floats.argtypes = [_u32, _u32]
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    _lib = lib
    return lib


def exported_symbols() -> list[str]:
    return ["dfhip_abi_version", "dfhip_last_error", "dfhip_march_rays_train_scratch_ints",
            "dfhip_grid_backward_default_parts", "dfhip_grid_backward_partial_floats",
            "dfhip_field_mlp_params", "dfhip_field_mlp_backward_parts",
            "dfhip_ray_head_partial_floats", "dfhip_march_rays_train_stage_floats",
            "dfhip_shading_partial_doubles", "dfhip_grid_backward_binned_tile",
            *_SIGS.keys()]


# ---------------------------------------------------------------- kernel timing
# Opt-in (bench.py): HIP events recorded on the launching stream around a
# region of the hot path, with the algorithmic bytes of that launch.

class _KernelTimer:
    def __init__(self):
        self.records = []  # (name, start_event, end_event, bytes or callable -> bytes)
        # name -> (fixed bytes, bytes per live row, live-row based?): the
        # region's byte model, to evaluate it at another run's row count
        self.models = {}

    def region(self, name, nbytes, live=None, per_row=0):
        if not callable(nbytes):
            self.models[name] = (nbytes, per_row, live is not None)
        return _Region(self, name, nbytes, live, per_row)


class _Region:
    __slots__ = ("timer", "name", "nbytes", "e0", "live", "per_row")

    def __init__(self, timer, name, nbytes, live, per_row):
        self.timer, self.name, self.nbytes = timer, name, nbytes
        self.live, self.per_row = live, per_row

    def __enter__(self):
        if self.live is not None:
            # snapshot the device-side row count (read when the records are
            # summarised, never inside the timed stretch)
            snap, base, per_row = self.live.clone(), self.nbytes, self.per_row
            self.nbytes = lambda: base + per_row * int(snap.item())
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e0.record()
        return self

    def __exit__(self, *exc):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.timer.records.append((self.name, self.e0, e1, self.nbytes))


def record_bytes(nbytes):
    """Bytes of a timing record (resolves deferred, device-count-based sizes)."""
    return nbytes() if callable(nbytes) else nbytes


class _NoRegion:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_REGION = _NoRegion()
_timer = None


def set_kernel_timer(timer):
    """Install (or remove with None) a _KernelTimer; returns the previous one."""
    global _timer
    prev, _timer = _timer, timer
    return prev


def new_kernel_timer():
    return _KernelTimer()


def timing():
    """The installed _KernelTimer, or None."""
    return _timer


def timed(name, nbytes, live=None, per_row=0):
    """Context manager timing one launch region when a timer is installed.
    Algorithmic bytes = nbytes + per_row * live[0] when `live` (an int32
    device tensor holding a row count) is given, else nbytes."""
    return _NO_REGION if _timer is None else _timer.region(name, nbytes, live, per_row)


def call(name: str, *args) -> None:
    rc = getattr(load(), name)(*args)
    if rc != 0:
        msg = load().dfhip_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


# ---------------------------------------------------------------- tensor helpers

def ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def dtype_code(t: torch.Tensor, what: str) -> int:
    try:
        return _DTYPE[t.dtype]
    except KeyError:
        raise RuntimeError(f"{what} must be a floating tensor (float32/float16/bfloat16/float64), "
                           f"got {t.dtype}")


def check_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what} must be a CUDA tensor")


def check_contig(t: torch.Tensor, what: str) -> None:
    if not t.is_contiguous():
        raise RuntimeError(f"{what} must be a contiguous tensor")


def check_int(t: torch.Tensor, what: str) -> None:
    if t.dtype != torch.int32:
        raise RuntimeError(f"{what} must be an int tensor")


def checked(t: torch.Tensor, what: str, kind: str = "float") -> torch.Tensor:
    """CHECK_CUDA + CHECK_CONTIGUOUS + dtype check (reference gridencoder.cu:15-18)."""
    check_cuda(t, what)
    check_contig(t, what)
    if kind == "int":
        check_int(t, what)
    elif kind == "i64":
        if t.dtype != torch.int64:
            raise RuntimeError(f"{what} must be an int64 tensor")
    elif kind == "u8":
        if t.dtype != torch.uint8:
            raise RuntimeError(f"{what} must be a uint8 tensor")
    else:
        dtype_code(t, what)
    return t
