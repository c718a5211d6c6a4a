"""The C-ABI library builds, loads and exports every entry point that
include/dfhip.h declares (no compute calls: these run without a GPU)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "dfhip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dfhip_[A-Za-z0-9_]+)\s*\(", text)))


def test_header_declares_the_reference_surface():
    syms = declared_symbols()
    # one entry point per reference binding (bindings.cpp of the 4 extensions)
    for name in ["near_far_from_aabb", "sph_from_ray", "morton3D", "morton3D_invert", "packbits",
                 "march_rays_train", "composite_rays_train_forward",
                 "composite_rays_train_backward", "march_rays", "composite_rays",
                 "grid_encode_forward", "grid_encode_backward", "freq_encode_forward",
                 "freq_encode_backward", "sh_encode_forward", "sh_encode_backward"]:
        assert f"dfhip_{name}" in syms


def test_library_exports_every_declared_symbol():
    import _dfhip
    lib = _dfhip.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.dfhip_abi_version() == 1
    assert set(_dfhip.exported_symbols()) == set(declared_symbols())


def test_errors_are_reported_without_a_gpu():
    """Argument validation runs before any device work, so it is testable here."""
    import ctypes
    import _dfhip
    lib = _dfhip.load()
    rc = lib.dfhip_grid_encode_forward(0, None, None, None, None, 10, 7, 2, 16, 0.5, 16, None, 1, 0,
                                       None)
    assert rc == 1
    assert b"D must be 1, 2, 3, 4, or 5" in lib.dfhip_last_error()
    rc = lib.dfhip_grid_encode_forward(0, None, None, None, None, 10, 3, 3, 16, 0.5, 16, None, 1, 0,
                                       None)
    assert rc == 1 and b"C must be 1, 2, 4, or 8" in lib.dfhip_last_error()
    rc = lib.dfhip_sh_encode_forward(0, None, None, 10, 3, 9, None, None)
    assert rc == 1 and b"degree in [1, 8]" in lib.dfhip_last_error()
    rc = lib.dfhip_freq_encode_forward(None, 4, 3, 6, 40, None, None)
    assert rc == 1
    rc = lib.dfhip_grid_encode_backward_blc(1, 1, None, None, None, None, 10, 3, 1, 16, 0.5, 16,
                                            None, None, 1, 0, None)
    assert rc == 2  # f16 accumulation with odd C (the reference silently drops it)
    # empty batches are no-ops that touch no device state
    assert lib.dfhip_morton3D(None, 0, None, None) == 0
    # one total per workgroup of R rays (R = DFHIP_MARCH_RPB of the build, 1..16)
    totals = lib.dfhip_march_rays_train_scratch_ints(16384)
    rpb = 16384 // totals
    assert 1 <= rpb <= 16 and rpb * totals == 16384
    assert lib.dfhip_march_rays_train_scratch_ints(rpb) == 1
    assert lib.dfhip_march_rays_train_scratch_ints(rpb + 1) == 2
    assert lib.dfhip_march_rays_train_scratch_ints(0) == 1


def test_shims_raise_on_cpu_tensors():
    import torch
    import _raymarching
    t = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="CUDA tensor"):
        _raymarching.near_far_from_aabb(t, t, torch.zeros(6), 4, 0.2, torch.zeros(4), torch.zeros(4))
