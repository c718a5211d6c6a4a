"""The albedo SDS train step as a fixed sequence of native launches, without
autograd (captured once in a HIP graph by nerf/graph.py).

The reference step (nerf/utils.py:337-404 train_step + 693-715 backward /
optimizer, with NeRFRenderer.run_cuda renderer.py:446-559 and
network_grid.common_forward :76-87) is, in the autograd form of this
package, ~50 launches per 128x128 step: the native kernels plus ~30 small
torch kernels (RNG draws, the light direction, SDS glue, loss assembly,
gradient fills and adds).  On MI355X every launch costs ~5 us of GPU time
even inside a graph, so the glue alone was ~140 us of a ~1.2 ms step.  Here
the step is, with the same kernels and the same arithmetic:

  prologue (eager, one launch; csrc/step.hip): camera rays from the host
      pose, near/far, march noise, the synthetic SDS gradient w(t) * eps at
      pred_rgb, step counter = 0
  graph: march count / emit -> f16 table copy -> fused grid field ->
      compositing -> ray head (background MLP, mix, depth, mask) -> entropy
      loss -> ray head backward with the entropy gradient fused into the
      weights-sum gradient -> compositing backward -> field MLP backward ->
      binned embedding backward -> GradScaler + Adam (single GPU: the
      learning rates are device values the prologue writes each step;
      data-parallel: the graph ends at the embedding gradient, and the
      all-reduce and Adam follow eagerly)

Every launch sits in a _dfhip.timed region with its algorithmic bytes (the
regions are no-ops unless a kernel timer is installed, and the graph is
captured without one): bench.py's kernel-timing pass runs the same body
eagerly under a timer for the per-kernel and step-level roofline.

Gradients are bit-identical to the autograd step given the same draws
(tests/test_gpu_native_step.py): the loss scale enters exactly where
autograd puts it (the entropy term's upstream gradient is the scale; the SDS
gradient is not scaled, the reference quirk kept by Trainer.backward_only).

With trainer.fused_backward off the step keeps the reference's two backward
passes (SDS latents.backward, sd.py:115, then scaler.scale(loss).backward(),
utils.py:708): the compositing / field backwards run once per pass and the
second pass adds into the parameter gradients, as autograd accumulates them.

Under bf16 autocast (trainer.bf16, BASELINE configs[4]) the table, features,
activations, colours and their gradients are bf16 (csrc/fieldmlp.hip's and
csrc/shade.hip's bf16 instantiations, v_mfma_f32_16x16x32_bf16) and there is
no GradScaler (the entropy and orientation terms' upstream gradient is 1).

Applies to the albedo shading with the InjectedSDS guidance, the
reference's grid network (16 x 2 tiled grid, 32 -> 64 -> 64 -> 4 MLP), a
background MLP (bg_radius > 0) or a random background colour, and
lambda_opacity == 0 (the -O defaults); anything else keeps the autograd step.
"""
import ctypes

import numpy as np
import torch

import _dfhip
import _fieldmlp
import _gridencoder
import _raymarching
from _dfhip import call, ptr, stream


# shading -> dfhip_shading code (csrc/shade.hip); albedo needs no shading kernel
SHADINGS = {"albedo": 0, "textureless": 1, "lambertian": 2}
FD_EPS = 1e-2  # network_grid.py:90 finite_difference_normal epsilon


def eligible(trainer, shading):
    """True when NativeAlbedoStep reproduces trainer.train_step for `shading`."""
    from .sd import InjectedSDS
    m, opt = trainer.model, trainer.opt
    if shading not in SHADINGS or not isinstance(trainer.guidance, InjectedSDS):
        return False
    if shading != "albedo" and not trainer.fused_backward:
        return False  # the two-pass form is built for the albedo step only
    if not ((trainer.fp16 or getattr(trainer, "bf16", False)) and m.cuda_ray):
        return False
    if opt.lambda_opacity > 0:
        return False
    enc = getattr(m, "encoder", None)
    if enc is None or getattr(enc, "offsets_host", None) is None:
        return False
    if (enc.num_levels, enc.level_dim, enc.input_dim) != (16, 2, 3):
        return False
    layers = list(m.sigma_net.net)
    if len(layers) != 3 or layers[0].bias is None:
        return False
    if [tuple(l.weight.shape) for l in layers] != [(64, 32), (64, 64), (4, 64)]:
        return False
    if m.bg_radius > 0 and m.native_background_layers() is None:
        return False
    return all(p.is_cuda and p.dtype == torch.float32 for p in m.parameters())


class NativeAlbedoStep:
    """Buffers and launches of one train step at resolution H x W.

    shading "albedo" (the default), or "textureless" / "lambertian" with the
    ambient ratio: the finite-difference normals' six stencil evaluations are
    rows [M, 7 M) of the same field launches (csrc/shade.hip), so every
    per-sample field buffer holds 7 x the march capacity."""

    def __init__(self, trainer, H, W, shading="albedo", ratio=1.0):
        self.trainer = trainer
        m, opt = trainer.model, trainer.opt
        dev = trainer.device
        self.H, self.W = int(H), int(W)
        N = self.N = self.H * self.W
        self.max_steps = int(opt.max_steps)
        cap = self.cap = N * self.max_steps
        self.shading, self.ratio = shading, float(ratio)
        self.shade_code = SHADINGS[shading]
        self.rows_per = 1 if self.shade_code == 0 else 7  # field rows per march sample
        fcap = self.fcap = cap * self.rows_per            # field-row capacity
        self.lam_orient = float(opt.lambda_orient) if self.shade_code else 0.0
        self.dt_gamma = float(opt.dt_gamma)
        self.lam = float(opt.lambda_entropy)
        f32 = dict(device=dev, dtype=torch.float32)
        # field element type: f16 (fp16 autocast, -O) or bf16 (bf16 autocast, C5)
        self.elem = torch.bfloat16 if getattr(trainer, "bf16", False) else torch.float16
        f16 = dict(device=dev, dtype=self.elem)
        bf = self.elem == torch.bfloat16
        self._shade_fwd = "dfhip_shading_forward_bf16" if bf else "dfhip_shading_forward"
        self._shade_bwd = "dfhip_shading_backward_bf16" if bf else "dfhip_shading_backward"
        i32 = dict(device=dev, dtype=torch.int32)
        # prologue outputs (graph inputs)
        self.rays_o = torch.empty(N, 3, **f32)
        self.rays_d = torch.empty(N, 3, **f32)
        self.nears = torch.empty(N, **f32)
        self.fars = torch.empty(N, **f32)
        self.noises = torch.empty(N, **f32)
        self.g_image = torch.empty(3, N, **f32)  # d loss / d pred_rgb (channel-major)
        self.bg_layers = m.native_background_layers() if m.bg_radius > 0 else None
        self.bg_color = None if self.bg_layers is not None else torch.empty(N, 3, **f32)
        self.counter = torch.zeros(2, **i32)
        self.aabb = np.ascontiguousarray(m.aabb_train.detach().float().cpu().numpy())
        g = trainer.guidance
        self.alphas = g.alphas.detach().float().contiguous()
        self.t_range = (int(g.min_step), int(g.max_step))
        # march
        self.rays = torch.empty(N, 3, **i32)
        self.block_sums = torch.empty(_raymarching.march_rays_train_scratch_ints(N), **i32)
        self.xyzs = torch.empty(cap, 3, **f32)
        self.dirs = torch.empty(cap, 3, **f32)
        self.deltas = torch.empty(cap, 2, **f32)
        # the count pass keeps each sample here; the emit pass only copies
        self.stage = torch.empty(_raymarching.march_rays_train_stage_floats(N, self.max_steps),
                                 **f32)
        self.m_dev = self.counter[:1]
        # field
        enc = m.encoder
        self.encoder = enc
        self.L, self.C = enc.offsets.shape[0] - 1, enc.level_dim
        self.rows = enc.embeddings.shape[0]
        self.meta = (float(np.log2(enc.per_level_scale)), int(enc.base_resolution),
                     enc.gridtype_id, bool(enc.align_corners), enc.offsets_host)
        self.table = torch.empty(self.rows, self.C, **f16)
        # corner quads of the table (dfhip_grid_quads): the forward's gathers
        self.quads = torch.empty(self.rows, 4, device=dev, dtype=torch.int32)
        self.mlp = []
        for lin in m.sigma_net.net:
            self.mlp += [lin.weight, lin.bias]
        self.enc = torch.empty(fcap, self.L * self.C, **f16)
        # field rows: the samples, or (shading) each sample followed by its six
        # stencil points (csrc/shade.hip); the compositing reads self.sigma
        self.sigma = torch.empty(cap, **f32)
        self.albedo = torch.empty(fcap, 3, **f16)
        self.xyz_field, self.sigma_field = self.xyzs, self.sigma
        self.m_field = self.m_dev  # live field rows: M, or 7 M with the stencil
        if self.shade_code:
            self.xyz_field = torch.empty(fcap, 3, **f32)
            self.sigma_field = torch.empty(fcap, **f32)
            self.m7 = torch.zeros(1, **i32)
            self.m_field = self.m7
            self.light = torch.empty(3, **f32)
            self.color = torch.empty(cap, 3, **f16)
            self.normal = torch.empty(cap, 3, **f32)
            self.orient = torch.zeros((), **f32)
            self.orient_partial = torch.empty(
                int(_dfhip.load().dfhip_shading_partial_doubles(cap)), device=dev,
                dtype=torch.float64)
            self.grad_color = torch.empty(cap, 3, **f16)
        # compositing + head
        self.ws = torch.empty(N, **f32)
        self.depth = torch.empty(N, **f32)
        self.image = torch.empty(N, 3, **f32)
        self.out_image = torch.empty(3, N, **f32)
        self.out_depth = torch.empty(N, **f32)
        self.mask = torch.empty(N, dtype=torch.uint8, device=dev)
        self.loss = torch.zeros((), **f32)
        # backward
        self.grad_image = torch.empty(N, 3, **f32)
        self.grad_ws = torch.empty(N, **f32)
        self.head_partial = (torch.empty(int(_dfhip.load().dfhip_ray_head_partial_floats(N)),
                                         **f32) if self.bg_layers is not None else None)
        self.grad_sigma = torch.empty(cap, **f32)
        self.grad_albedo = torch.empty(fcap, 3, **f16)
        self.grad_sigma_field = (torch.empty(fcap, **f32) if self.shade_code
                                 else self.grad_sigma)
        self.d_enc = torch.empty(self.L, fcap, self.C, **f16)
        self.mlp_partial = torch.empty(_fieldmlp.backward_parts(fcap) * _fieldmlp.params_count(),
                                       **f32)
        # shaded steps: the embedding backward bins and walks each sample's
        # 7-point stencil as one group (trainer.stencil_bin False: the 7 M rows
        # one by one)
        self.stencil_bin = bool(self.shade_code) and bool(getattr(trainer, "stencil_bin", True))
        ne, nc, npf = _gridencoder.grid_backward_binned_scratch(
            cap if self.stencil_bin else fcap, enc.offsets_host, self.L, self.C,
            group=7 if self.stencil_bin else 1)
        # counts zeroed once: every binned call leaves them clean, so the
        # step's calls skip the clearing launch (BinnedOpts.kept_clean)
        self.bin_scratch = (torch.empty(ne, **i32), torch.zeros(nc, **i32),
                            torch.empty(npf, **f32))
        sc = trainer.scaler
        if sc.is_enabled() and sc._scale is None:
            sc._lazy_init_scale_growth_tracker(dev)  # what scaler.scale() does on first use
        self._ones = torch.ones(1, **f32)  # upstream gradient of the loss without a scaler
        # gradients live in persistent buffers, written in place every step:
        # views of one flat bucket, which the data-parallel all-reduce
        # reduces in place (nerf/utils.py flat_allreduce_)
        from .utils import flat_grad_bucket_
        self.grad_bucket = flat_grad_bucket_(m.parameters())
        # the reference's two backward passes (SDS, then the scaled loss)
        self.two_pass = not trainer.fused_backward
        if self.two_pass:
            self.d_enc2 = torch.empty_like(self.d_enc)
            self.zero_image = torch.zeros(N, 3, **f32)
            self.grad_ws2 = torch.empty(N, **f32)
            # pass 2's compositing gradients in buffers of their own, so both
            # passes' intermediates stay readable after the step (tests)
            self.grad_sigma2 = torch.empty(cap, **f32)
            self.grad_albedo2 = torch.empty(cap, 3, **f16)
            self._emb_launch2 = None
        self.params = [p for p in m.parameters() if p.requires_grad]
        self.grads = [(p, p.grad) for p in self.params]
        self._emb_launch = None
        # dfhip_binned_opts of the embedding backward (tools: a walk trace of
        # the eager twin; None = the library defaults the scratch is sized for)
        self.binned_opts = None
        # optimizer inside the graph (attach_optimizer): the learning rates
        # live on the device, written by the prologue launch every step
        self.lr_dev = torch.zeros(8, **f32)
        self.dp_world = None  # attach_allreduce: the exchange joins the step
        self.dp_group = None
        self.adam = None
        self._lr_source = None
        self.n_params = sum(p.numel() for p in self.params)

    def attach_optimizer(self, native_adam):
        """Run GradScaler + Adam (nerf/optim.py NativeAdamAmp) as the step's
        last launches, with device learning rates (captured in the graph)."""
        self.adam = native_adam.device_lr_launch(self.lr_dev)
        self._lr_source = native_adam.group_lrs

    def attach_allreduce(self, world_size, group=None):
        """Make the step's tail the data-parallel exchange: ONE in-place
        all-reduce of the flat gradient bucket (flat_allreduce_'s bucket form,
        the reference's DDP averaging, utils.py:200-202) then the 1/world
        scaling, before the attached optimizer (captured in the graph)."""
        self.dp_world = int(world_size)
        self.dp_group = group

    def allreduce_tail(self):
        """The attached exchange (a timed region: the bucket read and written)."""
        import torch.distributed as dist
        with _dfhip.timed("grad_allreduce", 8 * self.n_params):
            dist.all_reduce(self.grad_bucket, op=dist.ReduceOp.SUM, group=self.dp_group)
            self.grad_bucket.div_(self.dp_world)

    def optimizer_tail(self):
        """The attached optimizer step (a timed region: 28 B per parameter)."""
        with _dfhip.timed("adam", 28 * self.n_params):
            self.adam()

    # ------------------------------------------------------------ per step
    def prologue(self, pose, intrinsics, seed, step):
        """Rays, near/far, noise, the SDS gradient and counter reset from the
        host pose [4, 4] (or [1, 4, 4]) of this step (one eager launch)."""
        host = np.ascontiguousarray(np.asarray(pose, dtype=np.float32).reshape(-1, 4, 4)[0, :3, :4])
        fx, fy, cx, cy = (float(v) for v in intrinsics)
        lo, hi = self.t_range
        lrs = self._lr_source() if self._lr_source is not None else []
        lr_host = (ctypes.c_float * max(1, len(lrs)))(*lrs)
        N = self.N
        with _dfhip.timed("step_prologue", N * (24 + 8 + 4 + 12) +
                          (12 * N if self.bg_color is not None else 0)):
            call("dfhip_train_step_prologue_lr", host.ctypes.data, fx, fy, cx, cy, self.H,
                 self.W, self.aabb.ctypes.data, 0.2, int(seed) & 0xFFFFFFFFFFFFFFFF,
                 int(step) & 0xFFFFFFFFFFFFFFFF, 1, ptr(self.alphas), lo, hi, ptr(self.rays_o),
                 ptr(self.rays_d), ptr(self.nears), ptr(self.fars), ptr(self.noises),
                 ptr(self.bg_color), ptr(self.g_image), ptr(self.counter), lr_host, len(lrs),
                 ptr(self.lr_dev), stream())
        if self.shade_code:
            # the light direction (renderer.py:462-464), same (seed, step) key
            call("dfhip_shading_light", ptr(self.rays_o), int(seed) & 0xFFFFFFFFFFFFFFFF,
                 int(step) & 0xFFFFFFFFFFFFFFFF, ptr(self.light), stream())

    def body(self):
        """Forward and backward down to the feature / network gradients (the
        graph-captured part).  Returns the loss tensor.  Each launch is a
        timed region with its algorithmic bytes (fixed + per live row)."""
        m = self.trainer.model
        N, cap = self.N, self.cap
        sc = self.trainer.scaler
        scale = sc._scale if sc.is_enabled() else self._ones
        T, md, mf = _dfhip.timed, self.m_dev, self.m_field
        hb = 2 if self.elem in (torch.float16, torch.bfloat16) else 4  # colour element bytes
        S, Hb, gridtype, align, _ = self.meta
        rc = self.rows * self.C

        def quads():
            with T("grid_quads", rc * (4 + hb) + 16 * self.rows):
                _fieldmlp.grid_quads(self.encoder.embeddings.detach(), self.encoder.offsets, S,
                                     Hb, gridtype, align, self.table, self.quads)
        # march (raymarching.py:161-235, device count): rays + near/far +
        # noise + bitfield in, (ray, offset, count) + one 20-B stage row per
        # sample out; the emit copies the stage into xyz / dir / delta rows
        with T("march_rays_train_count", 48 * N + (m.density_bitfield.numel()), md, 20):
            _raymarching.march_rays_train_count_staged(
                self.rays_o, self.rays_d, m.density_bitfield, m.bound, self.dt_gamma,
                self.max_steps, N, m.cascade, m.grid_size, self.nears, self.fars, self.rays,
                self.counter, self.noises, self.block_sums, self.stage)
        # per-sample directions only for the shadings (the albedo step reads
        # rays_d per ray): 12 B per sample fewer written
        dirs = self.dirs if self.shade_code else None
        with T("march_rays_train_emit", 24 * N, md, 52 if dirs is not None else 40):
            _raymarching.march_rays_train_emit_staged(
                self.rays_d, self.max_steps, N, cap, self.xyzs, dirs, self.deltas,
                self.rays, self.block_sums, 0, self.stage)
        # field (grid.py:38-39 autocast table, network_grid.py:76-87); with a
        # shading, the six finite-difference stencil points of every sample are
        # field rows too (network_grid.py:90-114)
        quads()
        if self.shade_code:
            with T("shading_stencil", 0, md, 12 + 84):
                call("dfhip_shading_stencil", ptr(self.xyzs), ptr(self.m_dev), cap, FD_EPS,
                     float(m.bound), ptr(self.xyz_field), ptr(self.m7), stream())
        with T("grid_field_forward", rc * hb, mf, 12 + self.L * self.C * hb + 4 + 3 * hb):
            _fieldmlp.grid_field_forward(self.xyz_field, m.bound, self.table,
                                         self.encoder.offsets, S, Hb, gridtype, align, self.mlp,
                                         self.enc, self.sigma_field, self.albedo, self.m_field,
                                         quads=self.quads)
        rgb = self.albedo
        if self.shade_code:
            # normals, lambertian, colour, orientation loss (network_grid.py:116-144,
            # renderer.py:485-489)
            with T("shading_forward", 0, md, 28 + 3 * hb + 12 + 4 + 3 * hb + 12):
                call(self._shade_fwd, ptr(self.sigma_field), ptr(self.albedo),
                     ptr(self.dirs), ptr(self.light), self.ratio, FD_EPS, self.shade_code,
                     ptr(self.m_dev), cap, ptr(self.sigma), ptr(self.color), ptr(self.normal),
                     ptr(self.orient_partial), self.lam_orient, ptr(self.orient), None, stream())
            rgb = self.color
        # compositing (raymarching.py:238-269)
        with T("composite_rays_train_forward", 32 * N, md, 4 + 3 * hb + 8):
            _raymarching.composite_rays_train_forward_mixed(
                self.sigma, rgb, self.deltas, self.rays, cap, N, 1e-4, self.ws, self.depth,
                self.image)
        # ray head (renderer.py:536-551) and the entropy regulariser (utils.py:386-391)
        bw = self._bg_weights()
        # the injected SDS gradient does not depend on pred_rgb: with the
        # background network and the entropy term, the head's forward comes out
        # of its backward launch (the recomputed background, bit-identical)
        combined = (not self.two_pass and self.lam > 0 and bw[0] is not None
                    and bool(getattr(self.trainer, "combined_head", True)))
        if not combined:
            with T("ray_head_forward", 60 * N):
                call("dfhip_ray_head_forward", N, ptr(self.ws), ptr(self.depth), ptr(self.image),
                     ptr(self.rays_d), ptr(self.nears), ptr(self.fars), *[ptr(w) for w in bw],
                     ptr(self.bg_color), ptr(self.out_image), ptr(self.out_depth),
                     ptr(self.mask), stream())
        if self.two_pass:
            if self.lam > 0:
                call("dfhip_entropy_forward", N, ptr(self.ws), self.lam, ptr(self.loss),
                     stream())
            self._add_orient_loss()
            # backward: SDS gradient at pred_rgb (unscaled), entropy gradient x scale
            self._backward_two_pass(bw, scale)
            return self.loss
        gbw = self._bg_grads()
        head_args = (N, ptr(self.g_image), ptr(self.ws), ptr(self.rays_d), *[ptr(w) for w in bw],
                     ptr(self.bg_color), ptr(self.grad_image), ptr(self.grad_ws), None,
                     ptr(self.head_partial), *[ptr(g) for g in gbw])
        with T("ray_head_backward", 60 * N if not combined else 120 * N):
            if combined:
                call("dfhip_ray_head_forward_backward_entropy_loss", N, ptr(self.ws),
                     ptr(self.depth), ptr(self.image), ptr(self.rays_d), ptr(self.nears),
                     ptr(self.fars), *[ptr(w) for w in bw], ptr(self.out_image),
                     ptr(self.out_depth), ptr(self.mask), ptr(self.g_image), ptr(self.grad_image),
                     ptr(self.grad_ws), ptr(self.head_partial), *[ptr(g) for g in gbw],
                     ptr(scale), self.lam, ptr(self.loss), stream())
            elif self.lam > 0:
                # head backward + the entropy term's gradient (upstream: the
                # scale); the entropy loss itself (utils.py:386-391) comes out
                # of the same launches (dfhip_entropy_forward's value)
                call("dfhip_ray_head_backward_entropy_loss", *head_args, ptr(scale), self.lam,
                     ptr(self.loss), stream())
            else:
                call("dfhip_ray_head_backward", *head_args, stream())
        self._add_orient_loss()
        with T("composite_rays_train_backward", 44 * N, md, 4 + 3 * hb + 8 + 4 + 3 * hb):
            _raymarching.composite_rays_train_backward_mixed(
                self.grad_ws, self.grad_image, self.sigma, rgb, self.deltas, self.rays,
                self.ws, self.image, cap, N, 1e-4, self.grad_sigma,
                self.grad_color if self.shade_code else self.grad_albedo, False)
        if self.shade_code:
            # density / colour / orientation gradients -> the field rows' gradients
            with T("shading_backward", 0, md, 28 + 3 * hb + 12 + 4 + 3 * hb + 28 + 21 * hb):
                call(self._shade_bwd, ptr(self.sigma_field), ptr(self.albedo),
                     ptr(self.dirs), ptr(self.light), self.ratio, FD_EPS, self.shade_code,
                     ptr(self.m_dev), cap, ptr(self.grad_sigma), ptr(self.grad_color),
                     ptr(scale), self.lam_orient, ptr(self.grad_sigma_field),
                     ptr(self.grad_albedo), stream())
        from gridencoder.grid import _parts
        # features + density / albedo gradients + positions in, feature
        # gradients out (the weight gradients are per-workgroup partials)
        per_bwd = 2 * self.L * self.C * hb + 4 + 3 * hb + 12
        with T("field_mlp_backward", 4 * _fieldmlp.params_count(), mf, per_bwd):
            _fieldmlp.grid_field_backward(
                self.enc, self.xyz_field, m.bound, self.mlp, self.grad_sigma_field,
                self.grad_albedo, self.d_enc, self.mlp_partial, [p.grad for p in self.mlp],
                self.encoder.offsets, self.rows, S, Hb, gridtype, align, None, None,
                _parts(self.rows, self.C), self.m_field)
        return self.loss

    def _backward_two_pass(self, bw, scale):
        """Pass 1: the SDS gradient alone (pred_rgb -> head -> compositing ->
        field); pass 2: the scaled entropy loss alone (weights_sum ->
        compositing -> field, no image gradient), adding into the gradients."""
        m = self.trainer.model
        N, cap = self.N, self.cap
        S, Hb, gridtype, align, _ = self.meta
        from gridencoder.grid import _parts
        gbw = self._bg_grads()
        call("dfhip_ray_head_backward", N, ptr(self.g_image), ptr(self.ws), ptr(self.rays_d),
             *[ptr(w) for w in bw], ptr(self.bg_color), ptr(self.grad_image), ptr(self.grad_ws),
             None, ptr(self.head_partial), *[ptr(g) for g in gbw], stream())
        passes = [(self.grad_ws, self.grad_image, self.grad_sigma, self.grad_albedo, self.d_enc,
                   False)]
        if self.lam > 0:
            passes.append((self.grad_ws2, self.zero_image, self.grad_sigma2, self.grad_albedo2,
                           self.d_enc2, True))
        for i, (g_ws, g_img, g_sig, g_alb, d_enc, acc) in enumerate(passes):
            if i == 1:
                call("dfhip_entropy_backward", N, ptr(self.ws), ptr(scale), self.lam,
                     ptr(self.grad_ws2), stream())
            _raymarching.composite_rays_train_backward_mixed(
                g_ws, g_img, self.sigma, self.albedo, self.deltas, self.rays, self.ws,
                self.image, cap, N, 1e-4, g_sig, g_alb, False)
            _fieldmlp.grid_field_backward(
                self.enc, self.xyzs, m.bound, self.mlp, g_sig, g_alb, d_enc,
                self.mlp_partial, [p.grad for p in self.mlp], self.encoder.offsets, self.rows, S,
                Hb, gridtype, align, None, None, _parts(self.rows, self.C), self.m_dev,
                accumulate=acc)

    def embedding_backward(self):
        """Binned embedding-gradient scatter (eager, timed like the autograd
        path's deferred launch)."""
        self._emb_launchers()
        if self.stencil_bin:  # per sample: its position + 7 rows of feature gradients
            live, per = self.m_dev, 12 + 7 * self.L * self.C * 2
        else:
            live, per = self.m_field, 12 + self.L * self.C * 2
        with _dfhip.timed("grid_encode_backward", 4 * self.rows * self.C, live, per):
            self._emb_launch()
        if self.two_pass and self.lam > 0:
            if self._emb_launch2 is None:
                m = self.trainer.model
                S, Hb, gridtype, align, offsets_host = self.meta
                self._emb_launch2 = _gridencoder.binned_launcher(
                    self.d_enc2, self.xyzs, m.bound, self.encoder.offsets, offsets_host,
                    self.encoder.embeddings.grad, self.cap, self.m_dev, 3, self.C, self.L, S,
                    Hb, gridtype, align, *self.bin_scratch, accumulate=True,
                    opts=self._kept_clean_opts())
            with _dfhip.timed("grid_encode_backward", 4 * self.rows * self.C, self.m_dev, per):
                self._emb_launch2()

    def _emb_launchers(self):
        """The binned embedding backward's launcher (bin, walk and sum)."""
        if self._emb_launch is not None:
            return
        m = self.trainer.model
        S, Hb, gridtype, align, offsets_host = self.meta
        if self.stencil_bin:
            args = (self.d_enc, self.xyzs, m.bound, self.encoder.offsets, offsets_host,
                    self.encoder.embeddings.grad, self.cap, self.m_dev, 3, self.C, self.L, S, Hb,
                    gridtype, align, *self.bin_scratch)
            kw = {"stencil_eps": FD_EPS}
        else:
            args = (self.d_enc, self.xyz_field, m.bound, self.encoder.offsets, offsets_host,
                    self.encoder.embeddings.grad, self.fcap, self.m_field, 3, self.C, self.L, S,
                    Hb, gridtype, align, *self.bin_scratch)
            kw = {}
        kw["opts"] = self._kept_clean_opts()
        self._emb_launch = _gridencoder.binned_launcher(*args, **kw)

    def _kept_clean_opts(self):
        """The call's BinnedOpts (self.binned_opts or the defaults) with
        kept_clean set: the persistent counts scratch needs no fill launch."""
        o = self.binned_opts if self.binned_opts is not None else _gridencoder.BinnedOpts()
        o.kept_clean = 1 if getattr(self.trainer, "kept_clean_scratch", True) else 0
        return o

    def time_field(self, reps=5):
        """Eager re-launches of the last step's fused field forward and MLP
        backward on its own buffers (both overwrite their outputs), timed with
        events on torch's current stream (the launch stream): average
        microseconds of each and the live field rows.  Measurement only: the
        step's results are unchanged."""
        m = self.trainer.model
        S, Hb, gridtype, align, _ = self.meta
        from gridencoder.grid import _parts

        def fwd():
            _fieldmlp.grid_field_forward(self.xyz_field, m.bound, self.table,
                                         self.encoder.offsets, S, Hb, gridtype, align, self.mlp,
                                         self.enc, self.sigma_field, self.albedo, self.m_field,
                                         quads=self.quads)

        def bwd():
            _fieldmlp.grid_field_backward(
                self.enc, self.xyz_field, m.bound, self.mlp, self.grad_sigma_field,
                self.grad_albedo, self.d_enc, self.mlp_partial, [p.grad for p in self.mlp],
                self.encoder.offsets, self.rows, S, Hb, gridtype, align, None, None,
                _parts(self.rows, self.C), self.m_field)

        out = []
        for fn in (fwd, bwd):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) * 1e3 / reps)
        return out[0], out[1], int(self.m_field.item())

    def reattach(self):
        for p, g in self.grads:
            p.grad = g

    # ------------------------------------------------------------ helpers
    def _add_orient_loss(self):
        """loss += lambda_orient * orient (utils.py:398-400).  The entropy
        launch writes the loss fresh each step; without it (lambda_entropy ==
        0) the orientation term overwrites it, so no step adds onto the last."""
        if self.lam_orient <= 0:
            return
        if self.lam > 0:
            self.loss.add_(self.orient, alpha=self.lam_orient)
        else:
            torch.mul(self.orient, self.lam_orient, out=self.loss)

    def _bg_weights(self):
        if self.bg_layers is None:
            return [None] * 4
        l1, l2 = self.bg_layers
        return [l1.weight, l1.bias, l2.weight, l2.bias]

    def _bg_grads(self):
        if self.bg_layers is None:
            return [None] * 4
        return [w.grad for w in self._bg_weights()]
