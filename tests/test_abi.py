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
    assert set(_dfhip.exported_symbols()) == set(declared_symbols())


def test_abi_version_is_the_header_hash():
    """dfhip_abi_version() is the hash of the header the library was built
    from (dfhip_build.abi_hash), and load() checks it against the header."""
    import _dfhip
    from dfhip_build import abi_hash
    assert _dfhip.load().dfhip_abi_version() == abi_hash()


def test_stale_library_fails_to_load(tmp_path, monkeypatch):
    """A library built from another header raises ImportError at load()
    instead of being called with other argument lists (the round-5 r05a
    segfault: Python passed the new 13-argument scratch query to a library
    still built for 9 arguments, whose `opts` pointer then read the integer
    gridtype = 1)."""
    import _dfhip
    import dfhip_build
    other = tmp_path / "dfhip.h"
    other.write_bytes(dfhip_build.HEADER.read_bytes() + b"\n/* one more declaration */\n")
    saved = _dfhip._lib
    monkeypatch.setattr(dfhip_build, "HEADER", other)
    _dfhip._lib = None
    try:
        with pytest.raises(ImportError, match="built from another include/dfhip.h"):
            _dfhip.load()
    finally:
        _dfhip._lib = saved


def _c_kind(decl):
    """ctypes kind of one C parameter declaration of dfhip.h."""
    decl = decl.strip()
    if "*" in decl or decl.startswith("dfhip_stream_t"):
        return "ptr"
    base = decl.rsplit(None, 1)[0] if len(decl.split()) > 1 else decl
    base = base.replace("const ", "").strip()
    return {"int": "i32", "int32_t": "i32", "uint32_t": "u32", "float": "f32",
            "uint64_t": "u64", "double": "f64"}[base]


def declared_prototypes():
    text = (ROOT / "include" / "dfhip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|uint32_t|uint64_t|const char \*)\s*(dfhip_\w+)\s*\(([^)]*)\)\s*;",
                         text):
        args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = [_c_kind(a) for a in args]
    return out


def test_python_signatures_follow_the_header():
    """Every ctypes argument list in _dfhip._SIGS has the header's arity and
    parameter kinds (pointer, i32, u32, f32, u64), so Python and the header
    cannot drift apart unnoticed (the header in turn pins the library through
    the ABI hash)."""
    import ctypes
    import _dfhip
    kind = {ctypes.c_void_p: "ptr", ctypes.c_int: "i32", ctypes.c_uint32: "u32",
            ctypes.c_float: "f32", ctypes.c_uint64: "u64"}
    protos = declared_prototypes()
    assert set(_dfhip._SIGS) <= set(protos)
    for name, args in _dfhip._SIGS.items():
        assert [kind[a] for a in args] == protos[name], name


def test_binned_scratch_query_without_a_gpu():
    """dfhip_grid_backward_binned_scratch_opts (host only) for single samples
    and stencil groups, every walk form, NULL and non-NULL options, with the
    reference grid's offsets; bad groups and walk forms are errors."""
    import numpy as np
    import _gridencoder
    from gridencoder.grid import level_offsets
    pls = np.exp2(np.log2(2048 / 16) / 15)
    offs = level_offsets(16, 2, 3, 16, pls, 16, False)
    base = _gridencoder.grid_backward_binned_scratch(1 << 20, offs, 16, 2)
    tile = _gridencoder.grid_backward_binned_tile()
    assert tile == 1024
    for group in (1, 7):
        assert _gridencoder.grid_backward_binned_tile(group=group) == tile
        for opts in (None, _gridencoder.BinnedOpts(), *(_gridencoder.BinnedOpts(walk_mode=m)
                                                       for m in (-1, 0, 1))):
            for cap in (0, 1, 1023, 1024, 1 << 20):
                e, c, p = _gridencoder.grid_backward_binned_scratch(cap, offs, 16, 2, opts,
                                                                    group=group)
                tiles = max(1, -(-cap // tile))
                assert e > 0 and c >= tiles * 111 and p > 0
                assert e == (tiles * 111 * tile + 1) // 2  # 111 slices on this grid
            assert _gridencoder.grid_backward_binned_scratch(1 << 20, offs, 16, 2, opts,
                                                             group=group) == base
    # more walk workgroups per CU: more partial images
    more = _gridencoder.BinnedOpts(walk_groups_per_cu=6)
    assert _gridencoder.grid_backward_binned_scratch(1 << 20, offs, 16, 2, more)[2] > base[2]
    for bad in (dict(group=3), dict(opts=_gridencoder.BinnedOpts(walk_mode=2)),
                dict(opts=_gridencoder.BinnedOpts(walk_groups_per_cu=17))):
        with pytest.raises(RuntimeError, match="binned"):
            _gridencoder.grid_backward_binned_scratch(1024, offs, 16, 2, **bad)
    with pytest.raises(RuntimeError, match="layout"):
        _gridencoder.grid_backward_binned_scratch(1024, offs, 0, 2)


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
