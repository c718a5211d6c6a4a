"""Deterministic synthetic inputs shared by the parity tests and fixtures."""
import math

import numpy as np

import oracle

H_GRID = 128
AABB = np.array([-1, -1, -1, 1, 1, 1], np.float32)


def camera_rays(h, w, seed=0, radius=1.3, fovy=55.0):
    """Rays of one orbit camera looking at the origin (provider/get_rays math,
    float32): rays_o, rays_d [h*w, 3]."""
    r = np.random.default_rng(seed)
    c = r.normal(size=3)
    c = c / np.linalg.norm(c) * radius
    fwd = -c / np.linalg.norm(c)
    up0 = np.array([0.0, -1.0, 0.0])
    right = np.cross(fwd, up0)
    right /= np.linalg.norm(right)
    up = np.cross(right, fwd)
    up /= np.linalg.norm(up)
    focal = h / (2 * math.tan(math.radians(fovy) / 2))
    j, i = np.meshgrid(np.arange(h) + 0.5, np.arange(w) + 0.5, indexing="ij")
    dirs = np.stack([(i - w / 2) / focal, (j - h / 2) / focal, np.ones_like(i)], -1).reshape(-1, 3)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    rot = np.stack([right, up, fwd], -1)
    rays_d = (dirs @ rot.T).astype(np.float32)
    rays_o = np.repeat(c[None].astype(np.float32), rays_d.shape[0], 0)
    return rays_o, rays_d


def cell_centres(H=H_GRID):
    ax = np.arange(H)
    c = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    return c.astype(np.int32), (2 * c / (H - 1) - 1)


def sphere_grid(radius=0.5, noise=0.0, seed=0, H=H_GRID):
    """Density grid [1, H^3] in morton order: 20 inside the sphere, 0 outside,
    plus a fraction `noise` of random occupied cells."""
    coords, xyz = cell_centres(H)
    inside = np.linalg.norm(xyz, axis=1) < radius
    if noise > 0:
        inside |= np.random.default_rng(seed).random(inside.shape[0]) < noise
    grid = np.zeros(H ** 3, np.float32)
    grid[oracle.morton3D(coords)] = np.where(inside, 20.0, 0.0)
    return grid[None]


def sphere_bitfield(radius=0.5, noise=0.0, seed=0):
    return oracle.packbits(sphere_grid(radius, noise, seed), 1.0)


def march_inputs(h=128, w=128, seed=0, radius=0.5, noise=0.002, min_near=0.2):
    rays_o, rays_d = camera_rays(h, w, seed)
    nears, fars = oracle.near_far_from_aabb(rays_o, rays_d, AABB, min_near)
    noises = np.random.default_rng(seed + 100).random(rays_o.shape[0], dtype=np.float32)
    bf = sphere_bitfield(radius, noise, seed)
    return rays_o, rays_d, nears, fars, noises, bf
