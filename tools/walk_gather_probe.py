"""Round-6 probe for the stencil walk's inline-data idea (the round-5
verdict's item 4: the binning writing each entry's data inline so the walk
streams it instead of gathering it).  Two variant libraries of
csrc/gridbin.hip, patched here so the product source keeps no probe knobs:

  gradlocal  every gradient-row load of the walk reads the row of the same
             slot in the FIRST binning tile (s mod 1,024: 28 KB per level,
             L1 / L2 resident).  Positions, cells, flushes and LDS adds are
             unchanged, so the control flow is the product's and only the
             gradient gathers' misses are gone: the most an inline gradient
             could save.  Results wrong (values only).
  alllocal   positions read the same way too (cells change: an upper bound on
             the gain of inlining everything, with fewer flushes / adds).

Both into lib/libdfhip_<name>.so, linked with the other objects of the last
build; compare `k_walk_flat` (textureless child) and `k_walk` (albedo) in
rocprofv3 kernel traces of the same bench child (tools/gpu_r06e.sh).
    python tools/walk_gather_probe.py"""
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "single-stable-dreamfusion_amd"
sys.path.insert(0, str(PKG))
import dfhip_build  # noqa: E402

BASE = (PKG / "csrc" / "gridbin.hip").read_text()

GRAD_SAT_OLD = "load_grad<grad_t, C>(gl + ((size_t)s * GROUP + (a < GROUP ? a : 0u)) * C, in.gs[0]);"
GRAD_SAT_NEW = "load_grad<grad_t, C>(gl + ((size_t)(s & 1023u) * GROUP + (a < GROUP ? a : 0u)) * C, in.gs[0]);"
GRAD_CEN_OLD = "load_group_grads<grad_t, C, GROUP>(gl + (size_t)s * GROUP * C, in.gs);"
GRAD_CEN_NEW = "load_group_grads<grad_t, C, GROUP>(gl + (size_t)(s & 1023u) * GROUP * C, in.gs);"
GROW_OLD = "gl + (size_t)(tbase + (v & kIdMask)) * GROUP * C);"
GROW_NEW = "gl + (size_t)((tbase + (v & kIdMask)) & 1023u) * GROUP * C);"
POS_OLD = "load_pos3<3>(inputs, s, in.xs);"
POS_NEW = "load_pos3<3>(inputs, s & 1023u, in.xs);"


def patch(src, pairs):
    for a, b in pairs:
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    return src


def build(name, src):
    tmp = Path(tempfile.mkdtemp(prefix="walkprobe_"))
    (tmp / "gridbin.hip").write_text(src)
    for h in (PKG / "csrc").glob("*.h"):
        (tmp / h.name).write_text(h.read_text().replace('"../../include/dfhip.h"', '"dfhip.h"'))
    obj = tmp / "gridbin.o"
    subprocess.run([dfhip_build.HIPCC, *dfhip_build.CFLAGS, "-c", str(tmp / "gridbin.hip"),
                    "-o", str(obj)], check=True)
    objs = [str(o) for o in sorted((PKG / "build").glob("*.o")) if o.name != "gridbin.o"]
    out = PKG / "lib" / f"libdfhip_{name}.so"
    subprocess.run([dfhip_build.HIPCC, f"--offload-arch={dfhip_build.ARCH}", "-shared", "-fPIC",
                    *objs, str(obj), "-o", str(out)], check=True)
    print(out)


if __name__ == "__main__":
    grad = [(GRAD_SAT_OLD, GRAD_SAT_NEW), (GRAD_CEN_OLD, GRAD_CEN_NEW), (GROW_OLD, GROW_NEW)]
    build("gradlocal", patch(BASE, grad))
    build("alllocal", patch(BASE, grad + [(POS_OLD, POS_NEW)]))
