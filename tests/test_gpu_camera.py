"""Native full-image camera rays (csrc/camera.hip) against the reference's
torch get_rays (nerf/utils.py:42-106, restated in nerf/utils.get_rays)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,W", [(128, 128), (64, 96), (1, 1), (33, 17)])
def test_native_rays_match_torch(gpu, H, W):
    from nerf.provider import rand_poses
    from nerf.utils import get_rays, get_rays_host_pose
    torch.manual_seed(H * 1000 + W)
    poses, _ = rand_poses(3, "cpu", radius_range=[1.0, 1.5])
    focal = H / (2 * np.tan(np.deg2rad(55.0) / 2))
    intr = np.array([focal, focal * 1.1, H / 2, W / 2])
    got = get_rays_host_pose(poses, intr, H, W, gpu)
    want = get_rays(poses.to(gpu), intr, H, W, -1)
    assert torch.equal(got["rays_o"], want["rays_o"].contiguous())
    # torch forms R d with a BLAS GEMM (its own summation order): ~1 ulp
    torch.testing.assert_close(got["rays_d"], want["rays_d"], rtol=0, atol=3e-7)


def test_dataset_collate_native(gpu):
    import main
    from nerf.provider import NeRFDataset
    opt = main.parse_opt(["--text", "x", "-O"])
    ds = NeRFDataset(opt, device=gpu, type="train", H=64, W=64, size=10)
    b = ds.collate([0])
    assert b["rays_o"].shape == (1, 64 * 64, 3) and b["rays_o"].is_cuda
    n = b["rays_d"].norm(dim=-1)
    torch.testing.assert_close(n, torch.ones_like(n), rtol=0, atol=1e-6)
    assert b["dir"].device.type == "cpu" and 0 <= int(b["dir"][0]) <= 5
