"""NeRF renderer (behavioural mirror of reference nerf/renderer.py).

`NeRFRenderer(opt)` keeps the reference's buffers (`aabb_train`, `aabb_infer`,
`density_grid`, `density_bitfield`, `step_counter` — checkpoint keys
unchanged), attributes (`bound`, `cascade`, `grid_size`, `mean_density`,
`mean_count`, `local_step`, ...) and methods (`run`, `run_cuda`,
`update_extra_state`, `render`, `reset_extra_state`), so a field written
against the reference (e.g. its nerf/network_grid.py) subclasses it unchanged.

The ray-marching ops it calls are the gfx950 kernels behind `raymarching`.
"""
import math

import torch
import torch.nn as nn

import raymarching
from .utils import custom_meshgrid, safe_normalize


def sample_pdf(bins, weights, n_samples, det=False):
    """Inverse-CDF importance sampling (reference renderer.py:15-49).
    bins [B, T], weights [B, T-1] -> new z values [B, n_samples]."""
    w = weights + 1e-5
    pdf = w / w.sum(-1, keepdim=True)
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), torch.cumsum(pdf, -1)], -1)
    if det:
        u = torch.linspace(0.5 / n_samples, 1.0 - 0.5 / n_samples, n_samples, device=w.device)
        u = u.expand(list(cdf.shape[:-1]) + [n_samples])
    else:
        u = torch.rand(list(cdf.shape[:-1]) + [n_samples], device=w.device)
    u = u.contiguous()
    hi_idx = torch.searchsorted(cdf, u, right=True)
    lo = (hi_idx - 1).clamp(min=0)
    hi = hi_idx.clamp(max=cdf.shape[-1] - 1)
    pair = torch.stack([lo, hi], -1)  # [B, n, 2]
    shape = [pair.shape[0], pair.shape[1], cdf.shape[-1]]
    cdf_g = torch.gather(cdf.unsqueeze(1).expand(shape), 2, pair)
    bins_g = torch.gather(bins.unsqueeze(1).expand(shape), 2, pair)
    span = cdf_g[..., 1] - cdf_g[..., 0]
    span = torch.where(span < 1e-5, torch.ones_like(span), span)
    frac = (u - cdf_g[..., 0]) / span
    return bins_g[..., 0] + frac * (bins_g[..., 1] - bins_g[..., 0])


class NeRFRenderer(nn.Module):
    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.bound = opt.bound
        self.cascade = 1 + math.ceil(math.log2(opt.bound))
        self.grid_size = 128
        self.cuda_ray = opt.cuda_ray
        self.min_near = opt.min_near
        self.density_thresh = opt.density_thresh
        self.bg_radius = opt.bg_radius

        b = opt.bound
        aabb = torch.FloatTensor([-b, -b, -b, b, b, b])
        self.register_buffer("aabb_train", aabb)
        self.register_buffer("aabb_infer", aabb.clone())

        if self.cuda_ray:
            cells = self.grid_size ** 3
            self.register_buffer("density_grid", torch.zeros([self.cascade, cells]))
            self.register_buffer("density_bitfield",
                                 torch.zeros(self.cascade * cells // 8, dtype=torch.uint8))
            self.mean_density = 0
            self.iter_density = 0
            self.register_buffer("step_counter", torch.zeros(16, 2, dtype=torch.int32))
            self.mean_count = 0
            self.local_step = 0
            self.last_counter = None
        # march_rays_train_dev instead of march_rays_train on the albedo train
        # path (set by the Trainer while it captures / replays the step graph)
        self.device_count_march = False
        # sync-free occupancy refresh on the GPU (False: the reference's torch ops)
        self.native_grid_update = True
        # native background mix / depth / mask (nerf/head.py; False: torch ops)
        self.native_head = True
        # fused persistent inference render when the field allows it (False: the
        # reference's march / field / composite host loop)
        self.native_infer = True
        # the fused renderer's gathers: through the corner-quad table (False:
        # 8-byte corner-pair gathers from the f16 table)
        self.infer_quads = True
        # its queue order: chunks of 2^infer_chunk_log2 consecutive rays, those
        # passing closest to the scene centre first (1, dfhip_render_ray_order),
        # those meeting the most occupied cells first (2,
        # dfhip_render_ray_order_occ), or pixel order (0)
        self.infer_order = 1
        self.infer_chunk_log2 = 6
        # the image width of the rays (row-major H x W, one or more images),
        # set by the caller: the queue's chunks are then 8 x 8 pixel tiles
        # (when 64-ray chunks apply and H is a multiple of 8), else 0: strips
        self.infer_tile_w = 0
        # eval frames: the background net runs on a side stream beside the
        # fused render (bit-identical; False: after it, in the head)
        self.infer_overlap_bg = True
        # generator of the density-grid jitter (None: torch's default)
        self.grid_generator = None
        # (nears, fars, xyzs, dirs, deltas, rays) of a march already run for
        # this train step (nerf/graph.py BucketedModuleStep), else None
        self.premarched = None

    # mean_density / mean_count: the sync-free grid refresh leaves them on the
    # device; they are read to the host only when somebody asks (checkpoint,
    # logging, the non-force_all_rays march), not every 16 steps.
    @property
    def mean_density(self):
        v = self.__dict__.get("_mean_density", 0)
        if torch.is_tensor(v):
            v = float(v)
            self.__dict__["_mean_density"] = v
        return v

    @mean_density.setter
    def mean_density(self, v):
        self.__dict__["_mean_density"] = v

    @property
    def mean_count(self):
        v = self.__dict__.get("_mean_count", 0)
        if torch.is_tensor(v):
            v = int(v)
            self.__dict__["_mean_count"] = v
        return v

    @mean_count.setter
    def mean_count(self, v):
        self.__dict__["_mean_count"] = v

    # field interface, implemented by the network subclass
    def forward(self, x, d):
        raise NotImplementedError()

    def density(self, x):
        raise NotImplementedError()

    def color(self, x, d, mask=None, **kwargs):
        raise NotImplementedError()

    def reset_extra_state(self):
        if not self.cuda_ray:
            return
        self.density_grid.zero_()
        self.mean_density = 0
        self.iter_density = 0
        self.step_counter.zero_()
        self.mean_count = 0
        self.local_step = 0

    @torch.no_grad()
    def export_mesh(self, path, resolution=None, S=128):
        """renderer.py:121-299: density on a resolution^3 lattice, isosurface at
        min(mean_density, density_thresh), `mesh.obj` under `path`.  mcubes /
        xatlas / nvdiffrast do not exist here: marching tetrahedra and vertex
        colours instead (nerf/mesh.py)."""
        from .mesh import export_mesh
        return export_mesh(self, path, resolution=resolution, S=S)

    def _bg(self, rays_d, bg_color):
        if self.bg_radius > 0:
            return self.background(rays_d.reshape(-1, 3))
        return 1 if bg_color is None else bg_color

    # ------------------------------------------------------------------ run()
    def run(self, rays_o, rays_d, num_steps=128, upsample_steps=128, light_d=None,
            ambient_ratio=1.0, shading="albedo", bg_color=None, perturb=False, **kwargs):
        """Coarse (uniform) + importance sampled rendering in plain torch
        (reference renderer.py:301-443).  rays_o, rays_d: [B, N, 3]."""
        prefix = rays_o.shape[:-1]
        rays_o = rays_o.contiguous().view(-1, 3)
        rays_d = rays_d.contiguous().view(-1, 3)
        N = rays_o.shape[0]
        device = rays_o.device
        results = {}
        aabb = self.aabb_train if self.training else self.aabb_infer

        nears, fars = raymarching.near_far_from_aabb(rays_o, rays_d, aabb, self.min_near)
        nears = nears.unsqueeze(-1)
        fars = fars.unsqueeze(-1)
        if light_d is None:
            light_d = safe_normalize(rays_o[0] + torch.randn(3, device=device, dtype=torch.float))

        z = torch.linspace(0.0, 1.0, num_steps, device=device).unsqueeze(0).expand((N, num_steps))
        z = nears + (fars - nears) * z
        sample_dist = (fars - nears) / num_steps
        if perturb:
            z = z + (torch.rand(z.shape, device=device) - 0.5) * sample_dist
        xyzs = rays_o.unsqueeze(-2) + rays_d.unsqueeze(-2) * z.unsqueeze(-1)
        xyzs = torch.min(torch.max(xyzs, aabb[:3]), aabb[3:])

        dens = {k: v.view(N, num_steps, -1) for k, v in self.density(xyzs.reshape(-1, 3)).items()}

        if upsample_steps > 0:
            with torch.no_grad():
                dz = z[..., 1:] - z[..., :-1]
                dz = torch.cat([dz, sample_dist * torch.ones_like(dz[..., :1])], dim=-1)
                alphas = 1 - torch.exp(-dz * dens["sigma"].squeeze(-1))
                trans = torch.cumprod(torch.cat([torch.ones_like(alphas[..., :1]),
                                                 1 - alphas + 1e-15], dim=-1), dim=-1)[..., :-1]
                weights = alphas * trans
                z_mid = z[..., :-1] + 0.5 * dz[..., :-1]
                new_z = sample_pdf(z_mid, weights[:, 1:-1], upsample_steps,
                                   det=not self.training).detach()
                new_xyzs = rays_o.unsqueeze(-2) + rays_d.unsqueeze(-2) * new_z.unsqueeze(-1)
                new_xyzs = torch.min(torch.max(new_xyzs, aabb[:3]), aabb[3:])
            new_dens = {k: v.view(N, upsample_steps, -1)
                        for k, v in self.density(new_xyzs.reshape(-1, 3)).items()}
            z, order = torch.sort(torch.cat([z, new_z], dim=1), dim=1)
            xyzs = torch.cat([xyzs, new_xyzs], dim=1)
            xyzs = torch.gather(xyzs, 1, order.unsqueeze(-1).expand_as(xyzs))
            for k in dens:
                both = torch.cat([dens[k], new_dens[k]], dim=1)
                dens[k] = torch.gather(both, 1, order.unsqueeze(-1).expand_as(both))

        dz = z[..., 1:] - z[..., :-1]
        dz = torch.cat([dz, sample_dist * torch.ones_like(dz[..., :1])], dim=-1)
        alphas = 1 - torch.exp(-dz * dens["sigma"].squeeze(-1))
        trans = torch.cumprod(torch.cat([torch.ones_like(alphas[..., :1]), 1 - alphas + 1e-15],
                                        dim=-1), dim=-1)[..., :-1]
        weights = alphas * trans

        dirs = rays_d.view(-1, 1, 3).expand_as(xyzs)
        sigmas, rgbs, normals = self(xyzs.reshape(-1, 3), dirs.reshape(-1, 3), light_d,
                                     ratio=ambient_ratio, shading=shading)
        rgbs = rgbs.view(N, -1, 3)
        if normals is not None:
            normals = normals.view(N, -1, 3)
            orient = weights.detach() * (normals * dirs).sum(-1).clamp(min=0) ** 2
            results["loss_orient"] = orient.sum(-1).mean()
            jitter = self.normal(xyzs + torch.randn_like(xyzs) * 1e-2).view(N, -1, 3)
            results["loss_smooth"] = (normals - jitter).abs().mean()

        weights_sum = weights.sum(dim=-1)
        depth = torch.sum(weights * ((z - nears) / (fars - nears)).clamp(0, 1), dim=-1)
        image = torch.sum(weights.unsqueeze(-1) * rgbs, dim=-2)
        image = image + (1 - weights_sum).unsqueeze(-1) * self._bg(rays_d, bg_color)

        results["image"] = image.view(*prefix, 3)
        results["depth"] = depth.view(*prefix)
        results["weights_sum"] = weights_sum
        results["mask"] = (nears < fars).reshape(*prefix)
        return results

    # ------------------------------------------------------------- run_cuda()
    def run_cuda(self, rays_o, rays_d, dt_gamma=0, light_d=None, ambient_ratio=1.0,
                 shading="albedo", bg_color=None, perturb=False, force_all_rays=False,
                 max_steps=1024, T_thresh=1e-4, **kwargs):
        """Occupancy-grid rendering (reference renderer.py:446-559)."""
        prefix = rays_o.shape[:-1]
        rays_o = rays_o.contiguous().view(-1, 3)
        rays_d = rays_d.contiguous().view(-1, 3)
        N = rays_o.shape[0]
        device = rays_o.device

        pre = self.premarched if self.training else None
        if pre is not None:
            nears, fars = pre[0], pre[1]
        else:
            # the train path passes no min_near -> the op's default 0.2 (renderer.py:458)
            nears, fars = raymarching.near_far_from_aabb(
                rays_o, rays_d, self.aabb_train if self.training else self.aabb_infer)
        if light_d is None and shading != "albedo":
            # the albedo field never reads the light; the reference draws it
            # anyway (renderer.py:466), which here would be seven tiny launches
            light_d = safe_normalize(rays_o[0] + torch.randn(3, device=device, dtype=torch.float))

        results = {}
        bg_net = None  # [N, 3] background colours computed ahead (eval, fused render)
        if self.training:
            if pre is None:
                counter = self.step_counter[self.local_step % 16]
                counter.zero_()
                self.local_step += 1
                self.last_counter = counter
            if pre is not None:
                # the march ran already (its count read on the host by the
                # caller, which keeps step_counter and local_step)
                xyzs, dirs, deltas, rays = pre[2:]
            elif self.device_count_march and force_all_rays and shading == "albedo":
                # no host sync: capacity-sized samples + device-side count (the
                # graph-captured train step); only the albedo path, whose
                # per-sample consumers all stop at the live count
                xyzs, dirs, deltas, rays = raymarching.march_rays_train_dev(
                    rays_o, rays_d, self.bound, self.density_bitfield, self.cascade,
                    self.grid_size, nears, fars, counter, perturb, dt_gamma, max_steps,
                    noises=getattr(self, "march_noises", None))
            else:
                noises = getattr(self, "march_noises", None)  # given draws (tests)
                xyzs, dirs, deltas, rays = raymarching.march_rays_train(
                    rays_o, rays_d, self.bound, self.density_bitfield, self.cascade,
                    self.grid_size, nears, fars, counter,
                    -1 if force_all_rays else self.mean_count,  # unused with force_all_rays
                    noises if (perturb and noises is not None) else perturb, 128, force_all_rays,
                    dt_gamma, max_steps)
            sigmas, rgbs, normals = self(xyzs, dirs, light_d, ratio=ambient_ratio, shading=shading)
            weights_sum, depth, image = raymarching.composite_rays_train(sigmas, rgbs, deltas, rays,
                                                                         T_thresh)
            if normals is not None:
                w = 1 - torch.exp(-sigmas)
                results["loss_orient"] = (w.detach() * (normals * dirs).sum(-1).clamp(min=0) ** 2).mean()
                jitter = self.normal(xyzs + torch.randn_like(xyzs) * 1e-2)
                results["loss_smooth"] = (normals - jitter).abs().mean()
        else:
            field = self.native_infer_field(shading, rays_o) if self.native_infer else None
            if field is not None:
                bg = self._background_async(rays_d, nears, fars, prefix, bg_color)
                weights_sum, depth, image = self._infer_fused(
                    rays_o, rays_d, nears, fars, field, perturb, dt_gamma, max_steps, T_thresh,
                    render_stream=bg[2] if bg else None)
                if bg:  # the background net ran beside the render
                    torch.cuda.current_stream().wait_event(bg[1])
                    bg[0].record_stream(torch.cuda.current_stream())
                    bg_net = bg[0].t().contiguous()
            else:
                weights_sum, depth, image = self._infer_loop(rays_o, rays_d, nears, fars, light_d,
                                                             ambient_ratio, shading, perturb,
                                                             dt_gamma, max_steps, T_thresh)

        results.update(self._compose(rays_d, nears, fars, weights_sum, depth, image, bg_color,
                                     prefix, bg_net))
        return results

    def _background_async(self, rays_d, nears, fars, prefix, bg_color):
        """The background MLP of the eval frame (network_grid.py:158-167) on a
        side stream, so it runs beside the fused render kernel instead of after
        it: dfhip_ray_head_forward with ws = 0 and image = 0 writes exactly
        bg = sigmoid(net(rays_d)) ([3, N]); _compose then mixes it in with the
        plain head (image + (1 - ws) * bg, the same f32 expression as the net
        head, so the frame is bit-identical).  Launched before the queue
        order, the net runs beside the order and the render.  Returns (bg,
        event, the render's stream), or None when the native head would not
        take the background net."""
        from . import head as _head
        if self.bg_radius <= 0 or not self.native_head or not self.infer_overlap_bg:
            return None
        if not (len(prefix) == 2 and prefix[0] == 1) or torch.is_grad_enabled():
            return None
        layers = self.native_background_layers()
        N = rays_d.shape[0]
        dev = rays_d.device
        if layers is None or not _head.head_eligible(nears, layers) or N == 0:
            return None
        z = self.__dict__.get("_bg_zeros")
        if z is None or z.numel() < 5 * N or z.device != dev:
            z = torch.zeros(5 * N, device=dev)  # ws, depth, image [N, 3]: zeros, kept
            self.__dict__["_bg_zeros"] = z
        pair = self.__dict__.get("_bg_streams")
        if pair is None or pair[0].device != dev:
            # two streams taken from torch's pool one after the other, the
            # render's and the net's: consecutive pool streams sit on
            # different hardware queues, so the net runs beside the render
            # (a stream that shares the render's queue runs after it)
            pair = (torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev))
            self.__dict__["_bg_streams"] = pair
            self.__dict__["_bg_stream"] = pair[1]
        side = pair[1]
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            side.wait_event(ready)
            out, _, _ = _head.ray_head(z[:N], z[N:2 * N], z[2 * N:5 * N].view(N, 3), rays_d,
                                       nears, fars, None, layers)
            done = torch.cuda.Event()
            done.record(side)
        for t in (rays_d, nears, fars, z):
            t.record_stream(side)
        return out, done, pair[0]

    def _compose(self, rays_d, nears, fars, weights_sum, depth, image, bg_color, prefix,
                 bg_net=None):
        """Background mix, depth normalisation, mask (renderer.py:536-551); on the
        GPU as the native ray head (nerf/head.py) when the shapes allow."""
        from . import head as _head
        net = self.bg_radius > 0 and bg_net is None
        layers = self.native_background_layers() if net else None
        bgc = bg_net if bg_net is not None else (None if net else bg_color)
        ok = (self.native_head and len(prefix) == 2 and prefix[0] == 1
              and (layers is not None if net else
                   (bgc is None or (torch.is_tensor(bgc) and bgc.shape == image.shape)))
              and _head.head_eligible(weights_sum, layers))
        if ok:
            out_image, out_depth, mask = _head.ray_head(weights_sum, depth, image, rays_d, nears,
                                                        fars, bgc, layers)
            # pred_rgb is stored channel-major: [1, N, 3] is a view of [3, N]
            return {"image": out_image.t().unsqueeze(0), "depth": out_depth.view(*prefix),
                    "weights_sum": weights_sum.reshape(*prefix), "mask": mask.view(*prefix)}
        image = image + (1 - weights_sum).unsqueeze(-1) * self._bg(rays_d, bg_color)
        # depth relative to the ray's near plane, normalised (renderer.py:547)
        return {"image": image.view(*prefix, 3),
                "depth": (torch.clamp(depth - nears, min=0) / (fars - nears)).view(*prefix),
                "weights_sum": weights_sum.reshape(*prefix),
                "mask": (nears < fars).reshape(*prefix)}

    def native_background_layers(self):
        """The background MLP's nn.Linear layers when the native ray head can
        evaluate it (frequency-encoded 39 -> 64 -> 3), else None (subclass hook)."""
        return None

    def native_infer_field(self, shading, x):
        """(encoder, [Linear] * 3) when the fused inference renderer can evaluate
        this field for `shading`, else None (subclass hook)."""
        return None

    def invalidate_infer_operands(self):
        """The parameters changed behind torch's back (native Adam, a graph
        replay, a checkpoint load): the next eval frame rebuilds its cached
        launch operands."""
        self.__dict__["_param_generation"] = self.__dict__.get("_param_generation", 0) + 1
        self.__dict__.pop("_infer_operands", None)

    def _infer_fused(self, rays_o, rays_d, nears, fars, field, perturb, dt_gamma, max_steps,
                     T_thresh, render_stream=None):
        """The inference loop below as ONE persistent launch (csrc/render.hip):
        march, grid field and compositing per ray with a device work queue, no
        host sync and no per-sample intermediates in HBM."""
        import _fieldmlp
        import numpy as np
        encoder, layers = field
        N = rays_o.shape[0]
        dev = rays_o.device
        weights_sum = torch.empty(N, dtype=torch.float32, device=dev)
        depth = torch.empty(N, dtype=torch.float32, device=dev)
        image = torch.empty(N, 3, dtype=torch.float32, device=dev)
        work = torch.empty(4, dtype=torch.int32, device=dev)
        noises = torch.rand(N, device=dev) if perturb else None
        # the field's launch operands (f32 weights, the f16 table and its corner
        # quads) are rebuilt only when a parameter changed: consecutive eval
        # frames reuse them.  Tensor versions miss the native optimizer (a
        # kernel writing through data_ptr, also inside a replayed graph), so
        # the trainer bumps param_generation after every optimizer step and
        # checkpoint load (invalidate_infer_operands)
        params = [encoder.embeddings] + [p for lin in layers for p in (lin.weight, lin.bias)]
        key = (self.__dict__.get("_param_generation", 0),
               *((p.data_ptr(), p._version) for p in params))
        cached = self.__dict__.get("_infer_operands")
        if cached is None or cached[0] != key:
            weights = []
            for lin in layers:
                weights += [lin.weight.detach().float().contiguous(),
                            lin.bias.detach().float().contiguous()]
            emb = encoder.embeddings.detach()
            if self.infer_quads:
                # the f16 cast and its corner quads in one launch (the field's
                # gathers then take two 16-byte loads per level)
                table = torch.empty(emb.shape, dtype=torch.half, device=dev)
                quads = torch.empty(emb.shape[0], 4, dtype=torch.int32, device=dev)
                _fieldmlp.grid_quads(emb.float().contiguous(), encoder.offsets,
                                     float(np.log2(encoder.per_level_scale)),
                                     int(encoder.base_resolution), encoder.gridtype_id,
                                     bool(encoder.align_corners), table, quads)
            else:
                table, quads = emb.to(torch.half).contiguous(), None
            cached = (key, weights, table, quads)
            self.__dict__["_infer_operands"] = cached
        _, weights, table, quads = cached
        import _dfhip
        # algorithmic bytes of the launch: rays in (o, d, near, far), outputs,
        # the f16 table and the bitfield once
        nbytes = N * (32 + 20) + table.numel() * 2 + self.density_bitfield.numel()
        # queue order: the chunks of 64 consecutive rays crossing the most of
        # the scene first (their rays do not then finish alone after the queue
        # ran dry: 0.38 -> 0.64 of the frame before it does)
        cl = int(self.infer_chunk_log2)
        while (N + (1 << cl) - 1) >> cl > 16384:  # the order kernel's chunk limit
            cl += 1
        tw = int(self.infer_tile_w)
        tile_w = tw if cl == 6 and tw > 0 and tw % 8 == 0 and N % (8 * tw) == 0 else 0
        occ = ((nears.float().contiguous(), fars.float().contiguous(), self.density_bitfield,
                self.bound, self.cascade, self.grid_size, max_steps)
               if self.infer_order == 2 else None)
        order = None
        if self.infer_order and N > 0:
            # rays in, one cost and one order entry per chunk out
            with _dfhip.timed("render_ray_order", N * 24 + 8 * ((N >> cl) + 1)):
                order = _fieldmlp.render_ray_order(rays_o.float().contiguous(),
                                                   rays_d.float().contiguous(), cl, occ=occ,
                                                   tile_w=tile_w)
        operands = (rays_o.float().contiguous(), rays_d.float().contiguous(),
                    nears.float().contiguous(), fars.float().contiguous())
        main = torch.cuda.current_stream()
        rs = render_stream if render_stream is not None else main
        if rs is not main:  # the render on its own stream (beside a side-stream job)
            rs.wait_stream(main)
        with torch.cuda.stream(rs), _dfhip.timed("render_rays_infer", nbytes):
            _fieldmlp.render_rays_infer(
                *operands, noises, self.bound,
                dt_gamma, max_steps, self.cascade, self.grid_size, self.density_bitfield,
                T_thresh, table, encoder.offsets, float(np.log2(encoder.per_level_scale)),
                int(encoder.base_resolution), encoder.gridtype_id, bool(encoder.align_corners),
                weights, weights_sum, depth, image, work, quads, order=order, chunk_log2=cl,
                tile_w=tile_w)
        if rs is not main:
            main.wait_stream(rs)
            for t in (*operands, weights_sum, depth, image, work, order, noises, table, quads,
                      *weights):
                if torch.is_tensor(t):
                    t.record_stream(rs)
        self.last_infer_work = work  # work[1] (+ 2^32 work[2]) = samples evaluated
        return weights_sum, depth, image

    def _infer_loop(self, rays_o, rays_d, nears, fars, light_d, ambient_ratio, shading, perturb,
                    dt_gamma, max_steps, T_thresh, n_step_max=8):
        """Alive-ray compaction loop of the inference render (renderer.py:496-532).
        n_step_max: the schedule's cap (8 in the reference; tests use 1)."""
        N = rays_o.shape[0]
        device = rays_o.device
        weights_sum = torch.zeros(N, dtype=torch.float32, device=device)
        depth = torch.zeros(N, dtype=torch.float32, device=device)
        image = torch.zeros(N, 3, dtype=torch.float32, device=device)
        rays_alive = torch.arange(N, dtype=torch.int32, device=device)
        rays_t = nears.clone()
        step = 0
        while step < max_steps:
            n_alive = rays_alive.shape[0]
            if n_alive <= 0:
                break
            n_step = max(min(N // n_alive, n_step_max), 1)
            xyzs, dirs, deltas = raymarching.march_rays(
                n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, self.bound,
                self.density_bitfield, self.cascade, self.grid_size, nears, fars, 128,
                perturb if step == 0 else False, dt_gamma, max_steps)
            sigmas, rgbs, _ = self(xyzs, dirs, light_d, ratio=ambient_ratio, shading=shading)
            raymarching.composite_rays(n_alive, n_step, rays_alive, rays_t, sigmas, rgbs, deltas,
                                       weights_sum, depth, image, T_thresh)
            rays_alive = rays_alive[rays_alive >= 0]
            step += n_step
        return weights_sum, depth, image

    # ------------------------------------------------------ occupancy grid
    @torch.no_grad()
    def update_extra_state(self, decay=0.95, S=128):
        """Refresh the density grid (EMA-max of jittered density queries) and
        re-pack the occupancy bitfield (reference renderer.py:562-615)."""
        if not self.cuda_ray:
            return
        if self.density_grid.is_cuda and S >= self.grid_size and self.native_grid_update:
            return self._update_extra_state_native(decay)
        tmp_grid = -torch.ones_like(self.density_grid)
        dev = self.density_bitfield.device
        axis = torch.arange(self.grid_size, dtype=torch.int32, device=dev).split(S)
        for xs in axis:
            for ys in axis:
                for zs in axis:
                    xx, yy, zz = custom_meshgrid(xs, ys, zs)
                    coords = torch.cat([xx.reshape(-1, 1), yy.reshape(-1, 1), zz.reshape(-1, 1)],
                                       dim=-1)
                    indices = raymarching.morton3D(coords).long()
                    xyzs = 2 * coords.float() / (self.grid_size - 1) - 1
                    for cas in range(self.cascade):
                        bound = min(2 ** cas, self.bound)
                        half = bound / self.grid_size
                        cas_xyzs = xyzs * (bound - half)
                        cas_xyzs += (self._grid_rand(cas_xyzs) * 2 - 1) * half
                        sig = self.density(cas_xyzs)["sigma"].reshape(-1).detach()
                        tmp_grid[cas, indices] = sig.to(tmp_grid.dtype)
        valid = self.density_grid >= 0
        self.density_grid[valid] = torch.maximum(self.density_grid[valid] * decay, tmp_grid[valid])
        self.mean_density = torch.mean(self.density_grid[valid]).item()
        self.iter_density += 1
        thresh = min(self.mean_density, self.density_thresh)
        self.density_bitfield = raymarching.packbits(self.density_grid, thresh,
                                                     self.density_bitfield)
        total_step = min(16, self.local_step)
        if total_step > 0:
            self.mean_count = int(self.step_counter[:total_step, 0].sum().item() / total_step)
        self.local_step = 0

    def _grid_rand(self, like):
        """Jitter draws of the grid refresh: from `grid_generator` when set (the
        Trainer seeds one identically on every rank, so data-parallel ranks
        keep identical occupancy grids without a collective),
        else torch's default generator (rand_like, renderer.py:593)."""
        gen = self.grid_generator
        if gen is None:
            return torch.rand_like(like)
        return torch.rand(like.shape, dtype=like.dtype, device=like.device, generator=gen)

    def _grid_points(self):
        """Cell-centre positions in [-1, 1] (x, y, z order of the reference's
        meshgrid) and their morton cell indices: constant, built once."""
        cached = self.__dict__.get("_grid_points_cache")
        dev = self.density_grid.device
        if cached is None or cached[0].device != dev:
            axis = torch.arange(self.grid_size, dtype=torch.int32, device=dev)
            xx, yy, zz = custom_meshgrid(axis, axis, axis)
            coords = torch.stack([xx.reshape(-1), yy.reshape(-1), zz.reshape(-1)], -1)
            indices = raymarching.morton3D(coords)
            xyzs = 2 * coords.float() / (self.grid_size - 1) - 1
            cached = (xyzs, indices)
            self.__dict__["_grid_points_cache"] = cached
        return cached

    @torch.no_grad()
    def _update_extra_state_native(self, decay):
        """update_extra_state with no host round trip (csrc/occupancy.hip): the
        same jittered queries (renderer.py:586-597), the EMA-max over valid
        cells and the mean / threshold / packbits on the device.  mean_density
        and mean_count stay device scalars until read."""
        import _dfhip
        xyzs, indices = self._grid_points()
        cells = self.grid_size ** 3
        acc = torch.zeros(2, dtype=torch.float64, device=xyzs.device)
        for cas in range(self.cascade):
            bound = min(2 ** cas, self.bound)
            half = bound / self.grid_size
            cas_xyzs = xyzs * (bound - half)
            cas_xyzs += (self._grid_rand(cas_xyzs) * 2 - 1) * half
            sig = self.density(cas_xyzs)["sigma"].reshape(-1).detach().float().contiguous()
            idx = indices if cas == 0 else indices + cas * cells
            _dfhip.call("dfhip_density_grid_ema", sig.data_ptr(), idx.data_ptr(), sig.numel(),
                        self.cascade * cells, float(decay), self.density_grid.data_ptr(),
                        acc.data_ptr(), _dfhip.stream())
        mean = torch.empty(1, dtype=torch.float32, device=xyzs.device)
        n_bytes = self.density_grid.numel() // 8
        _dfhip.call("dfhip_packbits_mean", self.density_grid.data_ptr(), n_bytes, acc.data_ptr(),
                    float(self.density_thresh), self.density_bitfield.data_ptr(),
                    mean.data_ptr(), _dfhip.stream())
        self.mean_density = mean[0]
        self.iter_density += 1
        total_step = min(16, self.local_step)
        if total_step > 0:
            # reference: int(sum / total_step); one native launch (torch's
            # reductions here would be first-use kernel loads mid-training)
            mc = torch.empty((), dtype=torch.int64, device=xyzs.device)
            _dfhip.call("dfhip_mean_count", self.step_counter.data_ptr(), total_step,
                        mc.data_ptr(), _dfhip.stream())
            self.mean_count = mc
        self.local_step = 0

    def render(self, rays_o, rays_d, staged=False, max_ray_batch=4096, **kwargs):
        """rays_o, rays_d: [B, N, 3] -> dict(image [B, N, 3], depth, weights_sum, ...)."""
        _run = self.run_cuda if self.cuda_ray else self.run
        B, N = rays_o.shape[:2]
        device = rays_o.device
        if not (staged and not self.cuda_ray):
            return _run(rays_o, rays_d, **kwargs)
        depth = torch.empty((B, N), device=device)
        image = torch.empty((B, N, 3), device=device)
        weights_sum = torch.empty((B, N), device=device)
        for b in range(B):
            for head in range(0, N, max_ray_batch):
                tail = min(head + max_ray_batch, N)
                r = _run(rays_o[b:b + 1, head:tail], rays_d[b:b + 1, head:tail], **kwargs)
                depth[b:b + 1, head:tail] = r["depth"]
                weights_sum[b:b + 1, head:tail] = r["weights_sum"]
                image[b:b + 1, head:tail] = r["image"]
        return {"depth": depth, "image": image, "weights_sum": weights_sum}
