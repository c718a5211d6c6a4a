"""Random orbit cameras (behavioural mirror of reference nerf/provider.py).

`rand_poses`, `circle_poses`, `get_view_direction` and `NeRFDataset` keep the
reference's signatures, RNG call order (torch then Python `random`) and
outputs: one full image of rays per batch (provider.py:202-236).
"""
import math
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


def _unit(v):
    n = math.sqrt(max(v[0] * v[0] + v[1] * v[1] + v[2] * v[2], 1e-20))
    return (v[0] / n, v[1] / n, v[2] / n)


def _cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def rand_poses_host(size, radius_range=(1, 1.5), theta_range=(0, 100), phi_range=(0, 360),
                    return_dirs=False, angle_overhead=30, angle_front=60, jitter=False,
                    uniform_sphere_rate=0.5):
    """rand_poses on the host in scalar Python (same distributions and formulas
    as provider.py:72-141, draws from Python's `random`; a few microseconds per
    camera instead of ~30 device ops and their syncs): poses [size, 4, 4] f32
    numpy, direction classes as a CPU long tensor (or None)."""
    t0, t1 = math.radians(theta_range[0]), math.radians(theta_range[1])
    p0, p1 = math.radians(phi_range[0]), math.radians(phi_range[1])
    overhead, front = math.radians(angle_overhead), math.radians(angle_front)
    rnd = random.random
    poses = np.zeros((size, 4, 4), np.float32)
    classes = []
    for b in range(size):
        radius = rnd() * (radius_range[1] - radius_range[0]) + radius_range[0]
        if rnd() < uniform_sphere_rate:
            u = _unit(((rnd() - 0.5) * 2.0, rnd(), (rnd() - 0.5) * 2.0))
            theta = math.acos(max(-1.0, min(1.0, u[1])))
            phi = math.atan2(u[0], u[2])
            if phi < 0:
                phi += 2 * math.pi
            center = (u[0] * radius, u[1] * radius, u[2] * radius)
        else:
            theta = rnd() * (t1 - t0) + t0
            phi = rnd() * (p1 - p0) + p0
            st = math.sin(theta)
            center = (radius * st * math.sin(phi), radius * math.cos(theta),
                      radius * st * math.cos(phi))
        target = (0.0, 0.0, 0.0)
        if jitter:
            center = tuple(c + (rnd() * 0.2 - 0.1) for c in center)
            target = tuple(random.gauss(0.0, 1.0) * 0.2 for _ in range(3))
        forward = _unit((target[0] - center[0], target[1] - center[1], target[2] - center[2]))
        right = _unit(_cross(forward, (0.0, -1.0, 0.0)))
        up = _cross(right, forward)
        if jitter:
            up = tuple(v + random.gauss(0.0, 1.0) * 0.02 for v in up)
        up = _unit(up)
        poses[b] = ((right[0], up[0], forward[0], center[0]),
                    (right[1], up[1], forward[1], center[1]),
                    (right[2], up[2], forward[2], center[2]),
                    (0.0, 0.0, 0.0, 1.0))
        if return_dirs:  # get_view_direction (same class order)
            cls = 0 if phi < front else (1 if phi < math.pi else (2 if phi < math.pi + front
                                                                    else 3))
            if theta <= overhead:
                cls = 4
            if theta >= math.pi - overhead:
                cls = 5
            classes.append(cls)
    dirs = torch.tensor(classes, dtype=torch.long) if return_dirs else None
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


class RayBatch(dict):
    """A collated camera batch whose full-image rays ("rays_o", "rays_d") are
    made on first access from the host pose ("pose", "intrinsics"): the
    graph-replayed train step writes them straight into its own input
    buffers instead (nerf/graph.py), eager callers see the usual dict."""

    def __missing__(self, key):
        if key in ("rays_o", "rays_d"):
            rays = get_rays_host_pose(self["pose"], self["intrinsics"], self["H"], self["W"],
                                      self["device"])
            self["rays_o"], self["rays_d"] = rays["rays_o"], rays["rays_d"]
            return self[key]
        raise KeyError(key)


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
        if native:  # rays made lazily from the host pose (RayBatch)
            return RayBatch(H=self.H, W=self.W, dir=dirs, device=self.device,
                            pose=np.asarray(poses, dtype=np.float32),
                            intrinsics=tuple(float(v) for v in intrinsics))
        rays = get_rays(poses, intrinsics, self.H, self.W, -1)
        return {"H": self.H, "W": self.W, "rays_o": rays["rays_o"], "rays_d": rays["rays_d"],
                "dir": dirs}

    def dataloader(self):
        return DataLoader(list(range(self.size)), batch_size=1, collate_fn=self.collate,
                          shuffle=self.training, num_workers=0)
