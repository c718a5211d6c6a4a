"""Host-side logic that needs no GPU: parameter layout, cameras, SDS math,
the data-parallel gradient exchange (gloo, 2 ranks), the SH table."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def test_grid_layout_and_param_count():
    import main
    from nerf.network_grid import NeRFNetwork
    opt = main.parse_opt(["--text", "x", "-O"])
    torch.manual_seed(0)
    net = NeRFNetwork(opt)
    assert net.encoder.embeddings.shape == (903480, 2)
    assert sum(p.numel() for p in net.parameters()) == 1816247
    keys = set(net.state_dict())
    for k in ["aabb_train", "aabb_infer", "density_grid", "density_bitfield", "step_counter",
              "encoder.embeddings", "encoder.offsets", "sigma_net.net.0.weight",
              "sigma_net.net.2.bias", "bg_net.net.1.weight"]:
        assert k in keys, k
    assert net.density_bitfield.numel() == 128 ** 3 // 8
    groups = net.get_params(1e-3)
    assert [g["lr"] for g in groups] == [1e-2, 1e-3, 1e-2, 1e-3]


def test_rays_and_poses_shapes():
    from nerf.provider import rand_poses, circle_poses, get_view_direction
    from nerf.utils import get_rays
    torch.manual_seed(0)
    poses, dirs = rand_poses(1, "cpu", return_dirs=True)
    assert poses.shape == (1, 4, 4) and dirs.shape == (1,)
    r = get_rays(poses, np.array([100.0, 100.0, 64.0, 64.0]), 128, 128)
    assert r["rays_o"].shape == (1, 16384, 3)
    np.testing.assert_allclose(r["rays_d"].norm(dim=-1).numpy(), 1.0, atol=1e-6)
    # rotation is orthonormal and the camera looks at the origin
    R = poses[0, :3, :3]
    np.testing.assert_allclose((R.T @ R).numpy(), np.eye(3), atol=1e-5)
    c = poses[0, :3, 3]
    np.testing.assert_allclose((R[:, 2] @ (-c / c.norm())).item(), 1.0, atol=1e-5)
    p2, _ = circle_poses("cpu", radius=1.8, theta=60, phi=0)
    np.testing.assert_allclose(p2[0, :3, 3].norm().item(), 1.8, atol=1e-6)
    cls = get_view_direction(torch.tensor([0.1, 1.5, 1.5, 3.0]), torch.tensor([0.0, 0.5, 3.5, 0.0]),
                             np.deg2rad(30), np.deg2rad(60))
    assert cls.tolist() == [4, 0, 2, 5]


def test_sds_math():
    from nerf.sd import scaled_linear_alphas_cumprod, add_noise, cfg_combine, SyntheticSDS
    a = scaled_linear_alphas_cumprod()
    betas = np.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000) ** 2
    np.testing.assert_allclose(a.numpy(), np.cumprod(1 - betas), rtol=1e-5)
    x, e = torch.randn(1, 4, 8, 8), torch.randn(1, 4, 8, 8)
    t = torch.tensor([500])
    np.testing.assert_allclose(add_noise(a, x, e, t).numpy(),
                               (a[500].sqrt() * x + (1 - a[500]).sqrt() * e).numpy(), rtol=1e-6)
    u, c = torch.randn(1, 4, 8, 8), torch.randn(1, 4, 8, 8)
    np.testing.assert_allclose(cfg_combine(torch.cat([u, c]), 100).numpy(),
                               (u + 100 * (c - u)).numpy(), rtol=1e-5, atol=1e-5)
    g = SyntheticSDS("cpu")
    tz = g.get_text_embeds(["a hamburger"], [""])
    assert tz.shape == (2, 77, 768)
    assert torch.equal(tz, g.get_text_embeds(["a hamburger"], [""]))  # deterministic
    img = torch.rand(1, 3, 64, 64, requires_grad=True)
    torch.manual_seed(3)
    lat, grad = g.sds_grad(tz, img)
    assert lat.shape == (1, 4, 64, 64) and grad.shape == lat.shape
    # train_step == backward of sds_grad's pair
    torch.manual_seed(3)
    assert g.train_step(tz, img) == 0
    g1 = img.grad.clone()
    img.grad = None
    torch.manual_seed(3)
    lat, grad = g.sds_grad(tz, img)
    lat.backward(grad)
    assert torch.allclose(img.grad, g1)


def _allreduce_worker(rank, world, port, out, bucket=False):
    import torch.distributed as dist
    from nerf.utils import _grad_bucket, flat_allreduce_, flat_grad_bucket_
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    lin = torch.nn.Linear(4, 3)
    emb = torch.nn.Parameter(torch.zeros(10, 2))
    params = list(lin.parameters()) + [emb]
    x = torch.full((2, 4), float(rank + 1))
    lin(x).sum().backward()
    emb.grad = torch.full_like(emb, float(rank))
    if bucket:
        # grads as views of one buffer (the native step): reduced in place
        flat = flat_grad_bucket_(params)
        assert _grad_bucket(params) is flat
        before = [p.grad for p in params]
        flat_allreduce_(params, world)
        assert all(p.grad is g for p, g in zip(params, before))
    else:
        flat_allreduce_(params, world)
    out[rank] = torch.cat([p.grad.reshape(-1) for p in params]).clone()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket", [False, True])
def test_flat_allreduce_gloo_two_ranks(bucket):
    port = 29500 + (os.getpid() % 1000) + (500 if bucket else 0)
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        out = m.dict()
        procs = [ctx.Process(target=_allreduce_worker, args=(r, 2, port, out, bucket))
                 for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
        g0, g1 = out[0], out[1]
    assert torch.equal(g0, g1)
    # weight grad of sum(Wx+b) is the column sums of x: mean over ranks of 2*(r+1)
    np.testing.assert_allclose(g0[:12].numpy(), np.full(12, 3.0))
    np.testing.assert_allclose(g0[12:15].numpy(), np.full(3, 2.0))
    np.testing.assert_allclose(g0[15:].numpy(), np.full(20, 0.5))


def test_sh_table_matches_oracle():
    """The generated kernel table (csrc/sh_table.h) equals the oracle's terms."""
    import re
    from pathlib import Path
    import oracle
    text = (Path(__file__).resolve().parents[1] / "single-stable-dreamfusion_amd" / "csrc" /
            "sh_table.h").read_text()
    rows = [list(map(lambda v: float(v.rstrip("f")), r.split(",")))
            for r in re.findall(r"\{([^{}]*)\},", text)]
    terms = {(idx, m): q for idx, m, q in oracle._sh_terms(8)}
    k = 0
    for l in range(8):
        for m in range(l + 1):
            q = terms[(l * l + l + m, m)]
            np.testing.assert_allclose(rows[k][:len(q)], q, rtol=1e-7)
            k += 1


def test_make_adam_keeps_generator_groups():
    """get_params() hands Adam generator-valued groups; make_adam must not
    consume them while deciding on the fused implementation."""
    import torch.nn as nn
    from nerf.utils import make_adam
    a, b = nn.Linear(3, 4), nn.Linear(4, 2)
    opt = make_adam([{"params": a.parameters(), "lr": 1e-2}, {"params": b.parameters(), "lr": 1e-3}],
                    betas=(0.9, 0.99), eps=1e-15)
    assert [len(g["params"]) for g in opt.param_groups] == [2, 2]
    assert opt.param_groups[0]["lr"] == 1e-2


def test_rand_poses_host():
    """Host (numpy) camera sampler: orthonormal look-at-origin poses, radius in
    range, view classes consistent with the torch get_view_direction."""
    import random

    import numpy as np
    import torch

    from nerf.provider import get_view_direction, rand_poses_host
    np.random.seed(0)
    random.seed(0)
    for _ in range(20):
        poses, dirs = rand_poses_host(4, radius_range=[1.0, 1.5], return_dirs=True)
        assert poses.shape == (4, 4, 4) and poses.dtype == np.float32
        R, c = poses[:, :3, :3], poses[:, :3, 3]
        np.testing.assert_allclose(R.transpose(0, 2, 1) @ R, np.tile(np.eye(3), (4, 1, 1)),
                                   atol=1e-5)
        r = np.linalg.norm(c, axis=1)
        assert np.all(r >= 1.0 - 1e-5) and np.all(r <= 1.5 + 1e-5)
        np.testing.assert_allclose(R[:, :, 2], -c / r[:, None], atol=1e-5)  # forward -> origin
        assert dirs.dtype == torch.int64 and int(dirs.min()) >= 0 and int(dirs.max()) <= 5
        thetas = torch.from_numpy(np.arccos(np.clip(c[:, 1] / r, -1, 1)).astype(np.float32))
        phis = np.arctan2(c[:, 0], c[:, 2])
        phis = torch.from_numpy(np.where(phis < 0, phis + 2 * np.pi, phis).astype(np.float32))
        want = get_view_direction(thetas, phis, np.deg2rad(30), np.deg2rad(60))
        assert (want == dirs).float().mean() >= 0.75  # boundary rounding may differ


def test_bench_launches_n_ranks_itself():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts two ranks itself
    (gloo self-test: no GPU work) and rank 0 reports n_gpus 2 / dp2 with
    bit-identical replicas after one all-reduced update."""
    import json
    import subprocess
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2",
                        "--launcher-selftest"], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["replicas_identical"]


def test_native_adam_unit_scale_only_for_bf16():
    """A disabled GradScaler (fp32 or bf16 training) takes the native
    unit-scale Adam only when the trainer asks for it (bf16); plain fp32 keeps
    torch Adam, which writes non-finite gradients where the native form skips."""
    import torch
    from nerf.optim import eligible
    p = torch.nn.Parameter(torch.zeros(4))
    opt = torch.optim.Adam([p], lr=1e-3)
    off = torch.amp.GradScaler("cuda", enabled=False)
    assert not eligible(opt, off)
    assert not eligible(opt, None, unit_scale=True)


def test_module_breakdown_counts_whole_steps(tmp_path):
    """bench._module_breakdown: per-step kernel time over whole steps between
    march count launches; the last step and anything after it are ignored."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "single-stable-dreamfusion_amd")]
    import bench
    rows = ["Kernel_Name,Start_Timestamp,End_Timestamp"]
    t = 0
    for step in range(5):
        for name, dur in (("void dfhip::rm::k_march_train_count<float, true>()", 50_000),
                          ("void dfhip::gb::k_bin_fast<true, 1u>()", 40_000),
                          ("__amd_rocclr_copyBuffer", 5_000)):
            rows.append(f"\"{name}\",{t},{t + dur}")
            t += dur + 1_000
    rows.append(f"\"at::native::reduce_kernel\",{t},{t + 900_000}")  # a post-run check
    f = tmp_path / "run_kernel_trace.csv"
    f.write_text("\n".join(rows) + "\n")
    bd = bench._module_breakdown([f], 3)
    assert bd["kernel_us_per_step"] == 95.0
    g = bd["groups_us_per_step"]
    assert g["march_rays_train"] == 50.0 and g["grid_encode_backward"] == 40.0
    assert g["runtime_copies_and_fills"] == 5.0 and "torch_elementwise_and_reductions" not in g
    assert bench._module_breakdown([f], 5) is None


def test_eval_background_side_stream_gating():
    """NeRFRenderer._background_async (the eval frame's background net beside
    the fused render) applies only to no-grad eval frames of one image on the
    GPU with the native head: here (CPU tensors, or grad enabled, or the
    option off, or no background net) it declines before any GPU call."""
    import main
    from nerf.network_grid import NeRFNetwork
    opt = main.parse_opt(["--text", "x", "-O"])
    torch.manual_seed(0)
    net = NeRFNetwork(opt).eval()
    assert net.bg_radius > 0 and net.infer_overlap_bg
    rays_d = torch.nn.functional.normalize(torch.randn(64, 3), dim=-1)
    nears, fars = torch.full((64,), 0.1), torch.full((64,), 2.0)
    with torch.no_grad():
        assert net._background_async(rays_d, nears, fars, (1, 64), None) is None  # CPU
        assert net._background_async(rays_d, nears, fars, (2, 32), None) is None  # two images
        net.infer_overlap_bg = False
        assert net._background_async(rays_d, nears, fars, (1, 64), None) is None
        net.infer_overlap_bg = True
        r = net.bg_radius
        net.bg_radius = 0.0
        assert net._background_async(rays_d, nears, fars, (1, 64), None) is None
        net.bg_radius = r
    assert net._background_async(rays_d, nears, fars, (1, 64), None) is None  # grad enabled
    assert "_bg_stream" not in net.__dict__ and "_bg_zeros" not in net.__dict__
