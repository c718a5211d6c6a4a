"""Round-6 probe for folding the embedding backward's binning into the fused
field forward (the round-5 verdict's item 5): binning needs a workgroup to
own whole 1,024-sample binning tiles (its LDS segment counters), so the
forward would have to walk its 16-sample MFMA tiles tile-owner by
tile-owner instead of strided over every resident wave.  This builds a
variant library whose k_field_fwd_fused does exactly that ownership walk
(no appends: a lower bound on a folded kernel's time) into
lib/libdfhip_foldprobe.so; compare its k_field_fwd_fused time against the
product library's in a rocprofv3 kernel trace of the same bench child.
    python tools/fold_probe.py   (then DFHIP_LIB=... for the child)"""
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "single-stable-dreamfusion_amd"
sys.path.insert(0, str(PKG))
import dfhip_build  # noqa: E402

src = (PKG / "csrc" / "fieldmlp.hip").read_text()
old_head = """    uint32_t tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    float xn[3] = {0.0f, 0.0f, 0.0f};"""
new_head = """    // probe: workgroup b owns binning tiles b, b + G, ... of 1,024 samples
    // (64 MFMA tiles each, wave w of 4 takes w, w + 4, ...)
    const uint32_t wv = threadIdx.x >> 6;
    uint32_t it = 0;
    auto tile_of = [&](uint32_t i) {
        return (blockIdx.x + (i >> 4) * gridDim.x) * 64u + wv + 4u * (i & 15u);
    };
    uint32_t tile = tile_of(0);
    float xn[3] = {0.0f, 0.0f, 0.0f};"""
old_loop = """    for (; tile < tiles; tile += waves) {"""
new_loop = """    for (; tile < tiles; tile = tile_of(++it)) {"""
old_next = """        const uint32_t nsample = (tile + waves) * 16 + c;"""
new_next = """        const uint32_t nsample = tile_of(it + 1) * 16 + c;"""
for a, b in ((old_head, new_head), (old_loop, new_loop), (old_next, new_next)):
    assert src.count(a) == 1, a
    src = src.replace(a, b)
# the launch: one workgroup per binning tile of the capacity, at most resident
old_launch = """    const uint32_t blocks = ceil_div(tiles, 4u) < fit ? ceil_div(tiles, 4u) : fit;
    k_field_fwd_fused<E, rgb_t, QUAD><<<blocks, 256, 0, s>>>("""
new_launch = """    const uint32_t btiles = ceil_div(tiles, 64u);
    const uint32_t blocks = btiles < fit ? btiles : fit;
    k_field_fwd_fused<E, rgb_t, QUAD><<<blocks, 256, 0, s>>>("""
assert src.count(old_launch) == 1
src = src.replace(old_launch, new_launch)
tmp = Path(tempfile.mkdtemp(prefix="foldprobe_"))
(tmp / "fieldmlp.hip").write_text(src)
for h in (PKG / "csrc").glob("*.h"):
    (tmp / h.name).write_text(h.read_text().replace('"../../include/dfhip.h"', '"dfhip.h"'))
obj = tmp / "fieldmlp.o"
subprocess.run([dfhip_build.HIPCC, *dfhip_build.CFLAGS, "-c", str(tmp / "fieldmlp.hip"), "-o",
                str(obj)], check=True)
objs = [str(o) for o in sorted((PKG / "build").glob("*.o")) if o.name != "fieldmlp.o"]
out = PKG / "lib" / "libdfhip_foldprobe.so"
subprocess.run([dfhip_build.HIPCC, f"--offload-arch={dfhip_build.ARCH}", "-shared", "-fPIC",
                *objs, str(obj), "-o", str(out)], check=True)
print(out)
