"""Random orbit cameras (behavioural mirror of reference nerf/provider.py).

`rand_poses`, `circle_poses`, `get_view_direction` and `NeRFDataset` keep the
reference's signatures, RNG call order (torch then Python `random`) and
outputs: one full image of rays per batch (provider.py:202-236).
"""
import random

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

from .utils import get_rays, get_rays_host_pose, safe_normalize


def get_view_direction(thetas, phis, overhead, front):
    """Direction class per camera: 0 front, 1 side, 2 back, 3 side, 4 overhead,
    5 bottom (provider.py:232-249)."""
    res = torch.zeros(thetas.shape[0], dtype=torch.long)
    res[phis < front] = 0
    res[(phis >= front) & (phis < np.pi)] = 1
    res[(phis >= np.pi) & (phis < (np.pi + front))] = 2
    res[phis >= (np.pi + front)] = 3
    res[thetas <= overhead] = 4
    res[thetas >= (np.pi - overhead)] = 5
    return res


def _look_at(centers, targets, jitter=False):
    forward = safe_normalize(targets - centers)
    up = torch.FloatTensor([0, -1, 0]).to(centers.device).unsqueeze(0).repeat(centers.shape[0], 1)
    right = safe_normalize(torch.cross(forward, up, dim=-1))
    noise = torch.randn_like(up) * 0.02 if jitter else 0
    up = safe_normalize(torch.cross(right, forward, dim=-1) + noise)
    poses = torch.eye(4, dtype=torch.float, device=centers.device).unsqueeze(0).repeat(
        centers.shape[0], 1, 1)
    poses[:, :3, :3] = torch.stack((right, up, forward), dim=-1)
    poses[:, :3, 3] = centers
    return poses


def rand_poses(size, device, radius_range=[1, 1.5], theta_range=[0, 100], phi_range=[0, 360],
               return_dirs=False, angle_overhead=30, angle_front=60, jitter=False,
               uniform_sphere_rate=0.5):
    """Random cameras looking at the origin (provider.py:72-141) -> poses [size, 4, 4]
    (cam2world), and direction classes if return_dirs."""
    theta_range = np.deg2rad(theta_range)
    phi_range = np.deg2rad(phi_range)
    angle_overhead = np.deg2rad(angle_overhead)
    angle_front = np.deg2rad(angle_front)

    radius = torch.rand(size, device=device) * (radius_range[1] - radius_range[0]) + radius_range[0]
    if random.random() < uniform_sphere_rate:
        unit = F.normalize(torch.stack([
            (torch.rand(size, device=device) - 0.5) * 2.0,
            torch.rand(size, device=device),
            (torch.rand(size, device=device) - 0.5) * 2.0,
        ], dim=-1), p=2, dim=1)
        thetas = torch.acos(unit[:, 1])
        phis = torch.atan2(unit[:, 0], unit[:, 2])
        phis[phis < 0] += 2 * np.pi
        centers = unit * radius.unsqueeze(-1)
    else:
        thetas = torch.rand(size, device=device) * (theta_range[1] - theta_range[0]) + theta_range[0]
        phis = torch.rand(size, device=device) * (phi_range[1] - phi_range[0]) + phi_range[0]
        centers = torch.stack([radius * torch.sin(thetas) * torch.sin(phis),
                               radius * torch.cos(thetas),
                               radius * torch.sin(thetas) * torch.cos(phis)], dim=-1)
    targets = 0
    if jitter:
        centers = centers + (torch.rand_like(centers) * 0.2 - 0.1)
        targets = targets + torch.randn_like(centers) * 0.2
    poses = _look_at(centers, targets, jitter)
    dirs = get_view_direction(thetas, phis, angle_overhead, angle_front) if return_dirs else None
    return poses, dirs


def _normalize_np(v):
    n = np.sqrt(np.maximum(np.sum(v * v, -1, keepdims=True), np.float32(1e-20)))
    return (v / n).astype(np.float32)


def rand_poses_host(size, radius_range=(1, 1.5), theta_range=(0, 100), phi_range=(0, 360),
                    return_dirs=False, angle_overhead=30, angle_front=60, jitter=False,
                    uniform_sphere_rate=0.5):
    """rand_poses on the host in numpy f32 (same distributions and formulas, a
    few microseconds instead of ~30 torch CPU ops): poses [size, 4, 4] f32
    numpy, direction classes as a CPU long tensor (or None)."""
    theta_range = np.deg2rad(theta_range)
    phi_range = np.deg2rad(phi_range)
    angle_overhead = np.deg2rad(angle_overhead)
    angle_front = np.deg2rad(angle_front)
    rnd = np.random.random_sample
    f32 = np.float32
    radius = (rnd(size).astype(f32) * f32(radius_range[1] - radius_range[0])
              + f32(radius_range[0]))
    if random.random() < uniform_sphere_rate:
        unit = _normalize_np(np.stack([(rnd(size).astype(f32) - f32(0.5)) * f32(2.0),
                                       rnd(size).astype(f32),
                                       (rnd(size).astype(f32) - f32(0.5)) * f32(2.0)], -1))
        thetas = np.arccos(unit[:, 1])
        phis = np.arctan2(unit[:, 0], unit[:, 2])
        phis = np.where(phis < 0, phis + f32(2 * np.pi), phis).astype(f32)
        centers = unit * radius[:, None]
    else:
        thetas = (rnd(size).astype(f32) * f32(theta_range[1] - theta_range[0])
                  + f32(theta_range[0]))
        phis = rnd(size).astype(f32) * f32(phi_range[1] - phi_range[0]) + f32(phi_range[0])
        centers = np.stack([radius * np.sin(thetas) * np.sin(phis), radius * np.cos(thetas),
                            radius * np.sin(thetas) * np.cos(phis)], -1).astype(f32)
    targets = np.zeros_like(centers)
    if jitter:
        centers = centers + (rnd(centers.shape).astype(f32) * f32(0.2) - f32(0.1))
        targets = targets + np.random.standard_normal(centers.shape).astype(f32) * f32(0.2)
    forward = _normalize_np(targets - centers)
    up = np.tile(np.array([[0, -1, 0]], f32), (size, 1))
    right = _normalize_np(np.cross(forward, up))
    noise = np.random.standard_normal(up.shape).astype(f32) * f32(0.02) if jitter else f32(0)
    up = _normalize_np(np.cross(right, forward) + noise)
    poses = np.tile(np.eye(4, dtype=f32)[None], (size, 1, 1))
    poses[:, :3, :3] = np.stack((right, up, forward), -1)
    poses[:, :3, 3] = centers
    dirs = None
    if return_dirs:  # get_view_direction in numpy (same class order)
        res = np.zeros(size, dtype=np.int64)
        res[phis < angle_front] = 0
        res[(phis >= angle_front) & (phis < np.pi)] = 1
        res[(phis >= np.pi) & (phis < (np.pi + angle_front))] = 2
        res[phis >= (np.pi + angle_front)] = 3
        res[thetas <= angle_overhead] = 4
        res[thetas >= (np.pi - angle_overhead)] = 5
        dirs = torch.from_numpy(res)
    return poses, dirs


def circle_poses(device, radius=1.25, theta=60, phi=0, return_dirs=False, angle_overhead=30,
                 angle_front=60):
    """One camera on the orbit at (theta, phi) degrees (provider.py:144-175)."""
    theta, phi = np.deg2rad(theta), np.deg2rad(phi)
    thetas = torch.FloatTensor([theta]).to(device)
    phis = torch.FloatTensor([phi]).to(device)
    centers = torch.stack([radius * torch.sin(thetas) * torch.sin(phis),
                           radius * torch.cos(thetas),
                           radius * torch.sin(thetas) * torch.cos(phis)], dim=-1)
    poses = _look_at(centers, torch.zeros_like(centers))
    dirs = (get_view_direction(thetas, phis, np.deg2rad(angle_overhead), np.deg2rad(angle_front))
            if return_dirs else None)
    return poses, dirs


class NeRFDataset:
    """Endless random-camera 'dataset' of full-image ray batches (provider.py:178-241)."""

    def __init__(self, opt, device, type="train", H=256, W=256, size=100):
        super().__init__()
        self.opt = opt
        self.device = device
        self.type = type
        self.H, self.W = H, W
        self.radius_range = opt.radius_range
        self.fovy_range = opt.fovy_range
        self.size = size
        self.training = self.type in ["train", "all"]
        # names swapped as in the reference (provider.py:194-195); equal at H == W
        self.cx = self.H / 2
        self.cy = self.W / 2

    def collate(self, index):
        """One full-image ray batch.  On the GPU the camera is drawn on the host
        (a handful of scalar ops; the reference draws it with device ops whose
        boolean-mask updates in get_view_direction synchronise every step) and
        the rays are made by one native launch (get_rays_host_pose)."""
        B = len(index)
        native = self.device is not None and torch.device(self.device).type == "cuda"
        pose_dev = "cpu" if native else self.device
        if self.training and native:
            poses, dirs = rand_poses_host(B, radius_range=self.radius_range,
                                          return_dirs=self.opt.dir_text,
                                          angle_overhead=self.opt.angle_overhead,
                                          angle_front=self.opt.angle_front,
                                          jitter=self.opt.jitter_pose,
                                          uniform_sphere_rate=self.opt.uniform_sphere_rate)
            poses = torch.from_numpy(poses)
            fov = random.random() * (self.fovy_range[1] - self.fovy_range[0]) + self.fovy_range[0]
        elif self.training:
            poses, dirs = rand_poses(B, pose_dev, radius_range=self.radius_range,
                                     return_dirs=self.opt.dir_text,
                                     angle_overhead=self.opt.angle_overhead,
                                     angle_front=self.opt.angle_front, jitter=self.opt.jitter_pose,
                                     uniform_sphere_rate=self.opt.uniform_sphere_rate)
            fov = random.random() * (self.fovy_range[1] - self.fovy_range[0]) + self.fovy_range[0]
        else:
            phi = (index[0] / self.size) * 360
            poses, dirs = circle_poses(pose_dev, radius=self.radius_range[1] * 1.2, theta=60,
                                       phi=phi, return_dirs=self.opt.dir_text,
                                       angle_overhead=self.opt.angle_overhead,
                                       angle_front=self.opt.angle_front)
            fov = (self.fovy_range[1] + self.fovy_range[0]) / 2
        focal = self.H / (2 * np.tan(np.deg2rad(fov) / 2))
        intrinsics = np.array([focal, focal, self.cx, self.cy])
        if native:
            rays = get_rays_host_pose(poses, intrinsics, self.H, self.W, self.device)
        else:
            rays = get_rays(poses, intrinsics, self.H, self.W, -1)
        return {"H": self.H, "W": self.W, "rays_o": rays["rays_o"], "rays_d": rays["rays_d"],
                "dir": dirs}

    def dataloader(self):
        return DataLoader(list(range(self.size)), batch_size=1, collate_fn=self.collate,
                          shuffle=self.training, num_workers=0)
