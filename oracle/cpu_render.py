"""Pure-PyTorch CPU restatement of the reference's --cuda_ray-off training step
— TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg, tests).

The reference has no runnable CPU renderer: its run() path still calls the
CUDA-only near_far_from_aabb, grid and frequency encoders.
This module restates, on CPU tensors:
  * raymarching.near_far_from_aabb          (raymarching.cu:91-145, vectorised)
  * GridEncoder forward (+autograd backward) (gridencoder.cu:75-313, tiled)
  * FreqEncoder                              (freqencoder.cu:28-94)
  * NeRFNetwork (grid backbone)              (nerf/network_grid.py:35-181)
  * NeRFRenderer.run + sample_pdf            (nerf/renderer.py:15-49, 301-443)
  * Trainer.train_step loss + Adam           (nerf/utils.py:337-404, main.py:128)
with the SDS guidance replaced by the same synthetic gradient stand-in as the
GPU bench (nerf/sd.py SyntheticSDS arithmetic).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


def near_far_from_aabb(rays_o, rays_d, aabb, min_near):
    inv = 1.0 / rays_d
    t0 = (aabb[:3] - rays_o) * inv
    t1 = (aabb[3:] - rays_o) * inv
    near = torch.minimum(t0, t1).nan_to_num(nan=-math.inf).amax(-1)
    far = torch.maximum(t0, t1).nan_to_num(nan=math.inf).amin(-1)
    miss = near > far
    near = torch.clamp(near, min=min_near)
    big = torch.finfo(torch.float32).max
    return torch.where(miss, big, near), torch.where(miss, big, far)


class TiledGridEncoder(nn.Module):
    """16-level tiled grid (align_corners=False) with torch autograd."""

    def __init__(self, num_levels=16, level_dim=2, base_resolution=16, log2_hashmap_size=16,
                 desired_resolution=2048):
        super().__init__()
        self.L, self.C, self.H = num_levels, level_dim, base_resolution
        pls = np.exp2(np.log2(desired_resolution / base_resolution) / (num_levels - 1))
        self.S = float(np.float32(np.log2(pls)))
        cap = 2 ** log2_hashmap_size
        offs, total = [], 0
        for l in range(num_levels):
            res = int(np.ceil(base_resolution * pls ** l))
            rows = int(np.ceil(min(cap, (res + 1) ** 3) / 8) * 8)
            offs.append(total)
            total += rows
        offs.append(total)
        self.offsets = offs
        self.embeddings = nn.Parameter(torch.empty(total, level_dim).uniform_(-1e-4, 1e-4))
        self.output_dim = num_levels * level_dim

    def forward(self, x, bound=1):
        x = (x + bound) / (2 * bound)
        B = x.shape[0]
        oob = ((x < 0) | (x > 1)).any(-1, keepdim=True)
        outs = []
        for l in range(self.L):
            e = np.float32(np.exp2(np.float64(np.float32(l) * np.float32(self.S))))
            scale = float(np.float32(e * np.float32(self.H) - np.float32(1)))
            res = int(np.ceil(scale)) + 1
            hs = self.offsets[l + 1] - self.offsets[l]
            pos = x * scale + 0.5
            cell = torch.floor(pos)
            frac = pos - cell
            cell = cell.long()
            acc = 0
            for k in range(8):
                bits = [(k >> d) & 1 for d in range(3)]
                w = torch.ones(B, dtype=x.dtype)
                idx = torch.zeros(B, dtype=torch.long)
                stride = 1
                for d in range(3):
                    w = w * (frac[:, d] if bits[d] else 1 - frac[:, d])
                    if stride <= hs:
                        idx = idx + (cell[:, d] + bits[d]) * stride
                        stride *= res + 1
                row = self.offsets[l] + torch.remainder(idx, hs)
                acc = acc + w[:, None] * self.embeddings[row]
            outs.append(acc)
        return torch.where(oob, torch.zeros(()), torch.cat(outs, -1))


def freq_encode(x, degree=6):
    parts = [x]
    for k in range(degree):
        parts += [torch.sin(x * 2.0 ** k), torch.cos(x * 2.0 ** k)]
    return torch.cat(parts, -1)


def _mlp(din, dout, dh, n):
    dims = [din] + [dh] * (n - 1) + [dout]
    layers = []
    for i in range(n):
        layers.append(nn.Linear(dims[i], dims[i + 1]))
        if i < n - 1:
            layers.append(nn.ReLU())
    return nn.Sequential(*layers)


class CPUNeRF(nn.Module):
    def __init__(self, bound=1.0, min_near=0.1):
        super().__init__()
        self.bound, self.min_near = bound, min_near
        self.encoder = TiledGridEncoder(desired_resolution=2048 * bound)
        self.sigma_net = _mlp(32, 4, 64, 3)
        self.bg_net = _mlp(39, 3, 64, 2)
        self.aabb = torch.tensor([-bound] * 3 + [bound] * 3)

    def density(self, x):
        h = self.sigma_net(self.encoder(x, bound=self.bound))
        g = 5 * torch.exp(-(x ** 2).sum(-1) / (2 * 0.2 ** 2))
        return torch.exp(h[..., 0] + g), torch.sigmoid(h[..., 1:])

    def run(self, rays_o, rays_d, num_steps=64, upsample_steps=64, perturb=True, det=False):
        """renderer.py:301-443 (albedo shading, bg net) -> image [N,3], weights_sum [N].
        det: sample_pdf's deterministic u (renderer.py:28-30, eval mode)."""
        N = rays_o.shape[0]
        nears, fars = near_far_from_aabb(rays_o, rays_d, self.aabb, self.min_near)
        nears, fars = nears[:, None], fars[:, None]
        z = nears + (fars - nears) * torch.linspace(0, 1, num_steps)[None]
        sd = (fars - nears) / num_steps
        if perturb:
            z = z + (torch.rand(z.shape) - 0.5) * sd
        xyz = torch.min(torch.max(rays_o[:, None] + rays_d[:, None] * z[..., None], self.aabb[:3]),
                        self.aabb[3:])
        sig, _ = self.density(xyz.reshape(-1, 3))
        sig = sig.view(N, num_steps)
        with torch.no_grad():
            dz = torch.cat([z[:, 1:] - z[:, :-1], sd.expand(N, 1)], -1)
            a = 1 - torch.exp(-dz * sig)
            w = a * torch.cumprod(torch.cat([torch.ones_like(a[:, :1]), 1 - a + 1e-15], -1), -1)[:, :-1]
            zm = z[:, :-1] + 0.5 * dz[:, :-1]
            wts = w[:, 1:-1] + 1e-5
            pdf = wts / wts.sum(-1, keepdim=True)
            cdf = torch.cat([torch.zeros_like(pdf[:, :1]), torch.cumsum(pdf, -1)], -1)
            if det:
                u = torch.linspace(0.5 / upsample_steps, 1 - 0.5 / upsample_steps,
                                   upsample_steps).expand(N, upsample_steps).contiguous()
            else:
                u = torch.rand(N, upsample_steps).contiguous()
            inds = torch.searchsorted(cdf, u, right=True)
            lo, hi = (inds - 1).clamp(min=0), inds.clamp(max=cdf.shape[-1] - 1)
            cl, ch = torch.gather(cdf, 1, lo), torch.gather(cdf, 1, hi)
            bl, bh = torch.gather(zm, 1, lo), torch.gather(zm, 1, hi)
            den = torch.where(ch - cl < 1e-5, torch.ones_like(cl), ch - cl)
            nz = bl + (u - cl) / den * (bh - bl)
            nxyz = torch.min(torch.max(rays_o[:, None] + rays_d[:, None] * nz[..., None],
                                       self.aabb[:3]), self.aabb[3:])
        nsig, _ = self.density(nxyz.reshape(-1, 3))
        z, order = torch.sort(torch.cat([z, nz], 1), 1)
        xyz = torch.gather(torch.cat([xyz, nxyz], 1), 1, order[..., None].expand(-1, -1, 3))
        sig = torch.gather(torch.cat([sig, nsig.view(N, upsample_steps)], 1), 1, order)
        dz = torch.cat([z[:, 1:] - z[:, :-1], sd.expand(N, 1)], -1)
        a = 1 - torch.exp(-dz * sig)
        w = a * torch.cumprod(torch.cat([torch.ones_like(a[:, :1]), 1 - a + 1e-15], -1), -1)[:, :-1]
        sig2, rgb = self.density(xyz.reshape(-1, 3))  # colour pass: self(xyzs, dirs, ...)
        rgb = rgb.view(N, -1, 3)
        ws = w.sum(-1)
        image = (w[..., None] * rgb).sum(-2)
        bg = torch.sigmoid(self.bg_net(freq_encode(rays_d)))
        image = image + (1 - ws)[:, None] * bg
        return image, ws


class CPUTrainStep:
    """One --cuda_ray-off SDS train step on CPU: render, SDS gradient, entropy
    regulariser, one backward, Adam.  guidance "injected" (the GPU bench's
    InjectedSDS: w(t) * N(0, 1) at pred_rgb) or "synthetic" (SDS arithmetic
    around stand-in VAE / UNet convolutions at 512^2)."""

    def __init__(self, H, W, seed=0, lr=1e-3, guidance="injected"):
        self.guidance = guidance
        torch.manual_seed(seed)
        self.H, self.W = H, W
        self.model = CPUNeRF()
        groups = [{"params": self.model.encoder.parameters(), "lr": lr * 10},
                  {"params": list(self.model.sigma_net.parameters()) +
                             list(self.model.bg_net.parameters()), "lr": lr}]
        self.opt = torch.optim.Adam(groups, betas=(0.9, 0.99), eps=1e-15)
        betas = torch.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000) ** 2
        self.alphas = torch.cumprod(1 - betas, 0)
        g = torch.Generator().manual_seed(1234)
        self.enc_w = torch.randn(4, 3, 1, 1, generator=g) * 0.5
        self.eps_w = torch.randn(4, 4, 1, 1, generator=g) * 0.1

    def rays(self):
        c = F.normalize(torch.randn(3), dim=0) * (1 + 0.5 * torch.rand(()))
        fwd = -c / c.norm()
        right = F.normalize(torch.cross(fwd, torch.tensor([0.0, -1.0, 0.0]), dim=0), dim=0)
        up = torch.cross(right, fwd, dim=0)
        focal = self.H / (2 * math.tan(math.radians(55) / 2))
        j, i = torch.meshgrid(torch.arange(self.H) + 0.5, torch.arange(self.W) + 0.5, indexing="ij")
        d = torch.stack([(i - self.W / 2) / focal, (j - self.H / 2) / focal, torch.ones_like(i)], -1)
        d = F.normalize(d.reshape(-1, 3), dim=-1) @ torch.stack([right, up, fwd], -1).T
        return c.expand_as(d).contiguous(), d.contiguous()

    def step(self):
        rays_o, rays_d = self.rays()
        self.opt.zero_grad()
        image, ws = self.model.run(rays_o, rays_d)
        pred = image.view(1, self.H, self.W, 3).permute(0, 3, 1, 2)
        a = ws.clamp(1e-5, 1 - 1e-5)
        loss = 1e-4 * (-a * torch.log2(a) - (1 - a) * torch.log2(1 - a)).mean()
        if self.guidance == "injected":
            t = int(torch.randint(20, 981, ()))
            grad = (1 - self.alphas[t]) * torch.randn_like(pred)
            torch.autograd.backward([pred, loss], [grad, None])
            self.opt.step()
            return float(loss.detach())
        x = F.avg_pool2d(2 * F.interpolate(pred, (512, 512), mode="bilinear",
                                           align_corners=False) - 1, 8)
        lat = F.conv2d(x, self.enc_w) * 0.18215
        t = int(torch.randint(20, 981, ()))
        with torch.no_grad():
            noise = torch.randn_like(lat)
            noisy = self.alphas[t].sqrt() * lat + (1 - self.alphas[t]).sqrt() * noise
            eps = F.conv2d(noisy, self.eps_w)
            grad = (1 - self.alphas[t]) * (eps - noise)
        torch.autograd.backward([lat, loss], [grad, None])
        self.opt.step()
        return float(loss.detach())
