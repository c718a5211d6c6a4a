"""Per-workgroup timeline of the binned grid backward's walk (k_walk) on the
samples of a real 128x128 march: which levels' workgroups take how long, how
many entries each walks, and how the launch's span splits into zeroing,
walking and write-out.  python tools/walk_trace.py [--reps 3]"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd"), str(ROOT / "tests"),
          str(ROOT / "tools")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--radius", type=float, default=0.56)
    ap.add_argument("--mode", type=int, default=0, help="walk mode (0 per segment, 3 resolved)")
    args = ap.parse_args()
    import _dfhip
    import _gridencoder
    import raymarching
    from gridencoder.grid import level_offsets
    from scenes import march_inputs
    lib = _dfhip.load()
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    rays_o, rays_d, nears, fars, _, bf = march_inputs(128, 128, seed=0, radius=args.radius,
                                                      noise=0.0)
    o, d, ne, fa, b = map(T, (rays_o, rays_d, nears, fars, bf))
    counter = torch.zeros(2, dtype=torch.int32, device=dev)
    xyzs, _, _, _ = raymarching.march_rays_train(o, d, 1.0, b, 1, 128, ne, fa, counter, -1, True,
                                                 128, True, 0.0, 512)
    B = xyzs.shape[0]
    x01 = ((xyzs + 1) / 2).contiguous()
    pls = np.exp2(np.log2(2048 / 16) / 15)
    S = float(np.log2(pls))
    offs = level_offsets(16, 2, 3, 16, pls, 16, False).astype(np.int32)
    L = 16
    g = (torch.randn(L, B, 2, device=dev) * 0.01).half()
    gemb = torch.empty(int(offs[-1]), 2, device=dev)
    trace = torch.zeros(8 * 8192, dtype=torch.int64, device=dev)
    opts = _gridencoder.BinnedOpts(walk_mode=args.mode, trace=trace)
    ne_, nc, npf = _gridencoder.grid_backward_binned_scratch(B, offs, L, 2, opts)
    ent = torch.empty(ne_, dtype=torch.int32, device=dev)
    cnt = torch.empty(nc, dtype=torch.int32, device=dev)
    part = torch.empty(npf, device=dev)
    ot = T(offs)
    for rep in range(args.reps + 1):
        trace.zero_()
        _gridencoder.grid_encode_backward_binned(g, x01, 0.0, ot, offs, gemb, B, None, 3, 2, L,
                                                 S, 16, 1, False, ent, cnt, part, opts=opts)
        torch.cuda.synchronize()
    report(trace, B, L, offs, shift=13)  # C = 2: 8,192-row slices


def report(trace, B, L, offs=None, shift=13):
    tr = trace.view(-1, 8).cpu().numpy()
    tr = tr[tr[:, 7] != 0]
    t0 = tr[:, 4].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731  wall clock: 100 MHz
    span = us(tr[:, 7].max())
    dur = (tr[:, 7] - tr[:, 4]) / 100.0
    plan = (tr[:, 5] - tr[:, 4]) / 100.0
    print(f"B={B} walk workgroups={len(tr)} span={span:.1f} us")
    print(f"workgroup duration mean {dur.mean():.1f} max {dur.max():.1f} min {dur.min():.1f} us; "
          f"plan mean {plan.mean():.2f} us; start max {us(tr[:, 4]).max():.1f} us")
    print(f"entries/workgroup mean {tr[:, 3].mean():.0f} max {tr[:, 3].max()}")
    # where the workgroups ran (trace column 1: XCC id << 32 | HW_ID)
    xcc = (tr[:, 1] >> 32).astype(np.int64)
    hw = (tr[:, 1] & 0xFFFFFFFF).astype(np.int64)
    cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 0x1) << 4) | (((hw >> 13) & 0x7) << 5)
    print("per XCC: workgroups / busy us (sum of durations) / last end us / CUs used")
    for x in np.unique(xcc):
        sel = xcc == x
        print(f"  xcc {x}: {int(sel.sum())} / {dur[sel].sum():.0f} / {us(tr[sel, 7]).max():.1f} / "
              f"{len(np.unique(cu[sel]))}")
    order = np.argsort(-dur)[:16]
    for i in order:
        print(f"  slow wg: bin {tr[i, 0]} parts {tr[i, 2]} xcc {tr[i, 1] >> 32} entries "
              f"{tr[i, 3]} dur {dur[i]:.1f} us start {us(tr[i, 4]):.1f}")
    ends = np.sort(us(tr[:, 7]))
    print("end-time quantiles (us):", [round(float(np.quantile(ends, q)), 1)
                                      for q in (0.1, 0.25, 0.5, 0.75, 0.9, 1.0)])
    print(f"total entries {tr[:, 3].sum()} ({tr[:, 3].sum() / B:.2f} per sample)")
    rate = {}
    for i in range(len(tr)):
        rate.setdefault(int(tr[i, 0]), []).append(tr[i, 3] / dur[i])
    print("bin: mean entries/us over its workgroups (ascending, first 12)")
    print("  " + "  ".join(f"{b}:{np.mean(v):.0f}" for b, v in
                           sorted(rate.items(), key=lambda kv: np.mean(kv[1]))[:12]))
    if offs is not None and shift:  # per-level entry rate of single-bin workgroups
        bin0 = [0]
        for lv in range(L):
            rows = int(offs[lv + 1] - offs[lv])
            bin0.append(bin0[-1] + ((rows - 1) >> shift) + 1)
        lvl = np.searchsorted(np.array(bin0), tr[:, 0], side="right") - 1
        one = np.ones(len(tr), bool)  # every workgroup walks one bin
        print("level: entries/us per workgroup (single-bin workgroups); max duration us")
        print("  " + "  ".join(f"{lv}:{(tr[one & (lvl == lv), 3] / dur[one & (lvl == lv)]).mean():.0f}"
                               for lv in range(L) if (one & (lvl == lv)).any()))
        print("  " + "  ".join(f"{lv}:{dur[one & (lvl == lv)].max():.0f}"
                               for lv in range(L) if (one & (lvl == lv)).any()))
        tot = {lv: int(tr[lvl == lv, 3].sum()) for lv in range(L)}
        print("level: entries, workgroups")
        print("  " + "  ".join(f"{lv}:{tot[lv]}/{int((lvl == lv).sum())}" for lv in range(L)))


if __name__ == "__main__":
    main()
