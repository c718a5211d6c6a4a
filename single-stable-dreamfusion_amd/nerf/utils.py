"""Camera rays, seeding and the SDS training loop (behavioural mirror of the
train-step parts of reference nerf/utils.py: get_rays :42-106, Trainer
:151-968 restricted to train_step / train_one_epoch / train / checkpoints).

Training-loop differences from the reference, each switchable:

* fused_backward (default on): the SDS latent gradient and the scaled
  regulariser loss are back-propagated in ONE autograd pass
  (`torch.autograd.backward([latents, scaler.scale(loss)], [grad, None])`).
  The reference runs two passes over the whole render graph
  (`latents.backward(grad, retain_graph=True)` in sd.py:115, then
  `scaler.scale(loss).backward()` in utils.py:708); the parameter gradients
  are the same sum, computed with one grid-backward scatter instead of two.
  The reference quirk that the SDS gradient is not multiplied by the scaler's
  scale (then divided by it in scaler.step) is kept in both modes.
* multi-GPU: one process per GPU; the trainable gradients are flattened into
  one buffer and all-reduced (RCCL over xGMI) before scaler.step, so every
  rank takes the same GradScaler skip decision.  No DDP wrapper (the
  reference's DDP path, utils.py:200-202, is dead code).
* loss.item() is not read every step (it is a host sync); losses are summed on
  the device and read once per epoch.
"""
import glob
import math
import os
import random
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def custom_meshgrid(*args):
    return torch.meshgrid(*args, indexing="ij")


def safe_normalize(x, eps=1e-20):
    return x / torch.sqrt(torch.clamp(torch.sum(x * x, -1, keepdim=True), min=eps))


@torch.autocast("cuda", enabled=False)
def get_rays(poses, intrinsics, H, W, N=-1, error_map=None):
    """Pinhole rays through pixel centres (reference utils.py:42-106).
    poses [B, 4, 4] cam2world, intrinsics (fx, fy, cx, cy) -> rays_o, rays_d [B, H*W, 3]
    (or N random pixels when N > 0)."""
    device = poses.device
    B = poses.shape[0]
    fx, fy, cx, cy = intrinsics
    i, j = custom_meshgrid(torch.linspace(0, W - 1, W, device=device),
                           torch.linspace(0, H - 1, H, device=device))
    i = i.t().reshape([1, H * W]).expand([B, H * W]) + 0.5
    j = j.t().reshape([1, H * W]).expand([B, H * W]) + 0.5
    results = {}
    if N > 0:
        N = min(N, H * W)
        if error_map is None:
            inds = torch.randint(0, H * W, size=[N], device=device).expand([B, N])
        else:
            coarse = torch.multinomial(error_map.to(device), N, replacement=False)
            ix, iy = coarse // 128, coarse % 128
            sx, sy = H / 128, W / 128
            ix = (ix * sx + torch.rand(B, N, device=device) * sx).long().clamp(max=H - 1)
            iy = (iy * sy + torch.rand(B, N, device=device) * sy).long().clamp(max=W - 1)
            inds = ix * W + iy
            results["inds_coarse"] = coarse
        i = torch.gather(i, -1, inds)
        j = torch.gather(j, -1, inds)
        results["inds"] = inds
    zs = torch.ones_like(i)
    xs = (i - cx) / fx * zs
    ys = (j - cy) / fy * zs
    dirs = safe_normalize(torch.stack((xs, ys, zs), dim=-1))
    rays_d = dirs @ poses[:, :3, :3].transpose(-1, -2)
    rays_o = poses[..., :3, 3][..., None, :].expand_as(rays_d)
    results["rays_o"] = rays_o
    results["rays_d"] = rays_d
    return results


_RAYS_FN = None


def get_rays_host_pose(poses, intrinsics, H, W, device, out=None):
    """get_rays(poses, intrinsics, H, W, N=-1) for host-side poses [B, 4, 4]
    (numpy or CPU tensor): one native launch per pose (csrc/camera.hip), the
    pose passed by value, so the per-step camera needs neither a host->device
    copy nor a sync.  Returns {"rays_o", "rays_d"} [B, H*W, 3] f32 on `device`
    (written into `out` = (rays_o, rays_d) when given)."""
    import ctypes

    import _dfhip
    global _RAYS_FN
    if _RAYS_FN is None:
        _RAYS_FN = _dfhip.load().dfhip_get_rays
    fx, fy, cx, cy = (float(v) for v in intrinsics)
    host = np.ascontiguousarray(poses.numpy() if torch.is_tensor(poses) else poses,
                                dtype=np.float32)
    B = host.shape[0]
    if out is None:
        rays_o = torch.empty(B, H * W, 3, device=device)
        rays_d = torch.empty(B, H * W, 3, device=device)
    else:
        rays_o, rays_d = out
        if rays_o.shape != (B, H * W, 3) or rays_d.shape != (B, H * W, 3):
            raise RuntimeError("get_rays_host_pose: output buffers must be [B, H*W, 3]")
    stream = _dfhip.stream()
    step = H * W * 3 * 4
    for b in range(B):
        pose = (ctypes.c_float * 12)(*host[b, :3, :4].reshape(-1).tolist())
        rc = _RAYS_FN(ctypes.cast(pose, ctypes.c_void_p), fx, fy, cx, cy, H, W,
                      rays_o.data_ptr() + b * step, rays_d.data_ptr() + b * step, stream)
        if rc != 0:
            raise RuntimeError(f"dfhip_get_rays failed ({rc}): "
                               f"{_dfhip.load().dfhip_last_error().decode()}")
    return {"rays_o": rays_o, "rays_d": rays_d}


def seed_everything(seed):
    """utils.py seed_everything, minus PYTHONHASHSEED: the hash seed is fixed
    when the interpreter starts, so setting it here only reaches child
    interpreters (none on this path)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)


# ----------------------------------------------------------------------------
# data-parallel gradient exchange
# ----------------------------------------------------------------------------

def flat_grad_bucket_(params):
    """Make the .grad of every trainable parameter a view of ONE contiguous
    f32 buffer (in parameter order), so the gradient all-reduce runs in place
    on it (no cat before / copies after).  Current gradient values are kept.
    Returns the buffer (also kept on the first parameter)."""
    params = [p for p in params if p.requires_grad]
    total = sum(p.numel() for p in params)
    flat = torch.zeros(total, dtype=torch.float32, device=params[0].device)
    off = 0
    for p in params:
        n = p.numel()
        view = flat[off:off + n].view_as(p)
        if p.grad is not None:
            view.copy_(p.grad)
        p.grad = view
        off += n
    params[0]._dfhip_grad_bucket = flat
    return flat


def _grad_bucket(params):
    """The flat buffer when the grads of `params` are still its consecutive
    views (flat_grad_bucket_), else None."""
    flat = getattr(params[0], "_dfhip_grad_bucket", None)
    if flat is None:
        return None
    ptr, off = flat.data_ptr(), 0
    for p in params:
        g = p.grad
        if g is None or g.dtype != torch.float32 or g.data_ptr() != ptr + 4 * off:
            return None
        off += g.numel()
    return flat if off == flat.numel() else None


def flat_allreduce_(params, world_size, group=None):
    """Average the .grad of `params` over all ranks with ONE all-reduce of a
    flat buffer (7.27 MB for the grid network: one RCCL ring / tree over xGMI
    instead of one collective per tensor).  Missing grads count as zeros.
    When the grads are views of one bucket (flat_grad_bucket_, the native
    step) the all-reduce and the 1/world scaling run in place on it."""
    params = [p for p in params if p.requires_grad]
    if not params or (world_size <= 1 and not (dist.is_available() and dist.is_initialized())):
        return
    bucket = _grad_bucket(params)
    if bucket is not None:
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
        bucket.div_(world_size)
        return
    dev = params[0].device
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).float()
                      for p in params])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.div_(world_size)
    off = 0
    for p in params:
        n = p.numel()
        chunk = flat[off:off + n].view_as(p).to(p.dtype)
        if p.grad is None:
            p.grad = chunk.clone()
        else:
            p.grad.copy_(chunk)
        off += n
    assert off == flat.numel() and flat.device == dev


def make_adam(params, **kw):
    """torch.optim.Adam as the reference builds it (main.py: betas (0.9, 0.99),
    eps 1e-15), as the single-kernel fused implementation when every
    parameter is on the GPU: it takes GradScaler's scale and inf flag on the
    device, so scaler.step() needs no host synchronisation (the foreach
    Adam + GradScaler path reads found_inf on the host every step)."""
    groups = []
    for g in params:  # materialise generators (e.g. module.parameters() in get_params groups)
        groups.append(dict(g, params=list(g["params"])) if isinstance(g, dict) else g)
    flat = [p for g in groups for p in (g["params"] if isinstance(g, dict) else [g])]
    if flat and all(p.is_cuda for p in flat):
        kw.setdefault("fused", True)
    return torch.optim.Adam(groups, **kw)


class _EMA:
    """Exponential moving average of parameters (stand-in for torch_ema)."""

    def __init__(self, params, decay):
        self.params = [p for p in params if p.requires_grad]
        self.decay = decay
        self.shadow = [p.detach().clone() for p in self.params]

    @torch.no_grad()
    def update(self):
        for s, p in zip(self.shadow, self.params):
            s.mul_(self.decay).add_(p.detach(), alpha=1 - self.decay)

    def state_dict(self):
        return {"decay": self.decay, "shadow": self.shadow}

    def load_state_dict(self, state):
        self.decay = state["decay"]
        for s, v in zip(self.shadow, state["shadow"]):
            s.copy_(v)


class Trainer(object):
    def __init__(self, name, opt, model, guidance, criterion=None, optimizer=None, ema_decay=None,
                 lr_scheduler=None, metrics=[], local_rank=0, world_size=1, device=None,
                 mute=False, fp16=False, bf16=False, eval_interval=1, max_keep_ckpt=2, workspace="workspace",
                 best_mode="min", use_loss_as_metric=True, report_metric_at_train=False,
                 use_checkpoint="latest", use_tensorboardX=True, scheduler_update_every_step=False,
                 fused_backward=True, graph_step=False):
        self.name = name
        self.opt = opt
        self.mute = mute
        self.metrics = metrics
        self.local_rank = local_rank
        self.world_size = world_size
        self.workspace = workspace
        self.ema_decay = ema_decay
        self.fp16 = fp16
        # bf16 autocast (BASELINE configs[4], the C5 option; the reference has
        # fp16 only): no GradScaler, the native step runs its bf16 field
        self.bf16 = bool(bf16) and not fp16
        self.amp = bool(fp16) or self.bf16
        self.amp_dtype = torch.bfloat16 if self.bf16 else torch.float16
        self.best_mode = best_mode
        self.use_loss_as_metric = use_loss_as_metric
        self.report_metric_at_train = report_metric_at_train
        self.max_keep_ckpt = max_keep_ckpt
        self.eval_interval = eval_interval
        self.use_checkpoint = use_checkpoint
        self.use_tensorboardX = use_tensorboardX
        self.time_stamp = time.strftime("%Y-%m-%d_%H-%M-%S")
        self.scheduler_update_every_step = scheduler_update_every_step
        self.fused_backward = fused_backward
        # HIP-graph replay of albedo steps (nerf/graph.py)
        self.graph_step = graph_step
        # data parallelism inside the replayed native step (nerf/graph.py): the
        # flat RCCL all-reduce, the 1/world scaling and GradScaler + Adam are
        # captured with the step.  None: whenever a process group with the
        # nccl (RCCL) backend is up; False: all-reduce + Adam eagerly after
        # the replay; True: capture with any backend that supports it
        self.dp_in_graph = None
        self._graphs = {}
        # GradScaler + Adam as one native call (nerf/optim.py) when eligible
        self.native_optimizer = True
        # the albedo / shaded steps as the native launch sequence
        # (nerf/native_step.py) where it applies; False: the autograd body
        self.native_step = True
        # shaded native steps: the embedding backward bins and walks each
        # sample's 7-point finite-difference stencil as one group (False: the
        # 7 M rows one by one)
        self.stencil_bin = True
        # native steps: the embedding backward's counts scratch is kept clean
        # by every call (no clearing launch per step; BinnedOpts.kept_clean)
        self.kept_clean_scratch = True
        # native steps with the injected SDS gradient: the ray head's forward
        # and backward as one launch (dfhip_ray_head_forward_backward_entropy_loss)
        self.combined_head = True
        # graph-replayed steps through the reference-API modules (no native
        # step, model.fused_field False): the host-count march, then a graph
        # per sample-count bucket (nerf/graph.py BucketedModuleStep)
        self.module_buckets = True
        # entropy regulariser as one native kernel each way (nerf/head.py)
        self.native_losses = True
        self._native_opt = None
        # bench.py kernel timing: called with the GraphedTrainStep in place of
        # its replay (runs the eager twin of the captured launches)
        self.step_hook = None
        self.device = device if device is not None else torch.device(
            f"cuda:{local_rank}" if torch.cuda.is_available() else "cpu")

        model.to(self.device)
        self.model = model
        if world_size > 1 and dist.is_available() and dist.is_initialized():
            # one replica: rank 0's parameters and buffers on every rank
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, src=0)
        self._capture_stream = None
        if (self.device.type == "cuda" and dist.is_available() and dist.is_initialized()
                and dist.get_backend() == "nccl"):
            # the communicator's first collective, issued by every rank here
            # (not inside a step): the graph capture's dry run issues none, so
            # a capturing step and a replaying step both issue exactly one.
            # It runs on the stream the step graphs are captured on, so the
            # first collective that stream sees is not the captured one.
            self._capture_stream = torch.cuda.Stream(device=self.device)
            self._capture_stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._capture_stream):
                dist.all_reduce(torch.zeros(1, device=self.device))
            torch.cuda.current_stream().wait_stream(self._capture_stream)
        if getattr(model, "cuda_ray", False) and self.device.type == "cuda":
            # the density-grid jitter draws the same numbers on every rank, so
            # the occupancy grids stay identical without a collective
            model.grid_generator = torch.Generator(device=self.device).manual_seed(
                int(getattr(opt, "seed", 0) or 0))
        self.guidance = guidance
        if self.guidance is not None:
            for p in self.guidance.parameters():
                p.requires_grad = False
            self.prepare_text_embeddings()
        else:
            self.text_z = None
        if isinstance(criterion, nn.Module):
            criterion.to(self.device)
        self.criterion = criterion

        if optimizer is None:
            self.optimizer = make_adam(self.model.parameters(), lr=0.001, weight_decay=5e-4)
        else:
            self.optimizer = optimizer(self.model)
        if lr_scheduler is None:
            self.lr_scheduler = torch.optim.lr_scheduler.LambdaLR(self.optimizer, lambda e: 1)
        else:
            self.lr_scheduler = lr_scheduler(self.optimizer)
        self.ema = _EMA(self.model.parameters(), ema_decay) if ema_decay is not None else None
        self.scaler = torch.amp.GradScaler("cuda", enabled=self.fp16)

        self.epoch = 0
        self.global_step = 0
        self.local_step = 0
        self.stats = {"loss": [], "valid_loss": [], "results": [], "checkpoints": [],
                      "best_result": None}
        if len(metrics) == 0 or self.use_loss_as_metric:
            self.best_mode = "min"
        self._pending_sds = None

        self.log_ptr = None
        if self.workspace is not None:
            os.makedirs(self.workspace, exist_ok=True)
            self.log_path = os.path.join(workspace, f"log_{self.name}.txt")
            self.log_ptr = open(self.log_path, "a+")
            self.ckpt_path = os.path.join(self.workspace, "checkpoints")
            self.best_path = f"{self.ckpt_path}/{self.name}.pth"
            os.makedirs(self.ckpt_path, exist_ok=True)
        self.log(f"[INFO] Trainer: {self.name} | {self.time_stamp} | {self.device} | "
                 f"{'fp16' if self.fp16 else 'bf16' if self.bf16 else 'fp32'} | {self.workspace}")
        self.log(f"[INFO] #parameters: {sum(p.numel() for p in model.parameters() if p.requires_grad)}")
        if self.workspace is not None and self.use_checkpoint not in (None, "scratch"):
            if self.use_checkpoint == "latest":
                self.load_checkpoint()
            elif self.use_checkpoint == "latest_model":
                self.load_checkpoint(model_only=True)
            elif self.use_checkpoint == "best":
                self.load_checkpoint(self.best_path if os.path.exists(self.best_path) else None)
            else:
                self.load_checkpoint(self.use_checkpoint)

    # ------------------------------------------------------------------ misc
    def prepare_text_embeddings(self):
        if self.opt.text is None:
            self.log("[WARN] text prompt is not provided.")
            self.text_z = None
            return
        if not self.opt.dir_text:
            self.text_z = self.guidance.get_text_embeds([self.opt.text], [self.opt.negative])
            return
        self.text_z = []
        for d in ["front", "side", "back", "side", "overhead", "bottom"]:
            negative = f"{self.opt.negative}"
            if self.opt.suppress_face and d != "front":
                negative = (negative + ", " if negative else "") + "face"
            self.text_z.append(self.guidance.get_text_embeds([f"{self.opt.text}, {d} view"],
                                                             [negative]))

    def __del__(self):
        if getattr(self, "log_ptr", None):
            self.log_ptr.close()

    def log(self, *args, **kwargs):
        if self.local_rank != 0:
            return
        if not self.mute:
            print(*args)
        if self.log_ptr:
            print(*args, file=self.log_ptr)
            self.log_ptr.flush()

    # ------------------------------------------------------------ train step
    def pick_shading(self):
        """Shading of this step (utils.py:346-360): albedo during the first
        albedo_iters steps, then albedo / textureless / lambertian at 20/40/40 %."""
        if self.global_step < self.opt.albedo_iters:
            return "albedo", 1.0
        r = random.random()
        if r > 0.8:
            return "albedo", 1.0
        if r > 0.4:
            return "textureless", 0.1
        return "lambertian", 0.1

    def train_step(self, data, shading=None, ambient_ratio=None, text_z=None):
        """Render one random view, take the SDS step and assemble the
        regularisers (reference utils.py:337-404).  Returns
        (pred_rgb [B,3,H,W], pred_ws [B,1,H,W], loss).  shading / text_z are
        picked here (as the reference does) unless given."""
        rays_o, rays_d = data["rays_o"], data["rays_d"]
        B, N = rays_o.shape[:2]
        H, W = data["H"], data["W"]
        if shading is None:
            shading, ambient_ratio = self.pick_shading()
        bg_color = torch.rand((B * N, 3), device=rays_o.device)
        opt_kwargs = dict(vars(self.opt))
        outputs = self.model.render(rays_o, rays_d, staged=False, perturb=True, bg_color=bg_color,
                                    ambient_ratio=ambient_ratio, shading=shading,
                                    force_all_rays=True, **opt_kwargs)
        pred_rgb = outputs["image"].reshape(B, H, W, 3).permute(0, 3, 1, 2).contiguous()
        if text_z is None:
            text_z = self.text_z[data["dir"]] if self.opt.dir_text else self.text_z
        if self.fused_backward and hasattr(self.guidance, "sds_grad"):
            self._pending_sds = self.guidance.sds_grad(text_z, pred_rgb)
            loss = 0
        else:
            loss = self.guidance.train_step(text_z, pred_rgb)
        pred_ws = outputs["weights_sum"].reshape(B, 1, H, W)
        if self.opt.lambda_opacity > 0:
            loss = loss + self.opt.lambda_opacity * (pred_ws ** 2).mean()
        if self.opt.lambda_entropy > 0:
            if pred_ws.is_cuda and pred_ws.dtype == torch.float32 and self.native_losses:
                from .head import ray_entropy  # native fwd / bwd (csrc/head.hip)
                loss = loss + ray_entropy(pred_ws, self.opt.lambda_entropy)
            else:
                a = pred_ws.clamp(1e-5, 1 - 1e-5)
                ent = (-a * torch.log2(a) - (1 - a) * torch.log2(1 - a)).mean()
                loss = loss + self.opt.lambda_entropy * ent
        if self.opt.lambda_orient > 0 and "loss_orient" in outputs:
            loss = loss + self.opt.lambda_orient * outputs["loss_orient"]
        if self.opt.lambda_smooth > 0 and "loss_smooth" in outputs:
            loss = loss + self.opt.lambda_smooth * outputs["loss_smooth"]
        return pred_rgb, pred_ws, loss

    def backward_and_step(self, loss):
        """Back-propagate (fused or reference two-pass), exchange gradients across
        ranks and take the (scaled) optimizer step."""
        self.backward_only(loss)
        self.optimizer_step()

    def backward_only(self, loss):
        """The backward half of backward_and_step (captured in the step graph)."""
        scaled = self.scaler.scale(loss) if torch.is_tensor(loss) else None
        if self._pending_sds is not None:
            latents, grad = self._pending_sds
            self._pending_sds = None
            roots, grads = [latents], [grad]
            if scaled is not None:
                roots.append(scaled)
                grads.append(None)
            torch.autograd.backward(roots, grads)
        elif scaled is not None:
            scaled.backward()

    def native_adam(self):
        """The native GradScaler + Adam (nerf/optim.py) when it reproduces
        this trainer's optimizer step, else False."""
        if self._native_opt is None:
            from . import optim as _optim
            self._native_opt = (_optim.NativeAdamAmp(self.optimizer, self.scaler)
                                if self.native_optimizer and _optim.eligible(
                                    self.optimizer, self.scaler, unit_scale=self.bf16)
                                else False)
        return self._native_opt

    def graph_collective(self):
        """True when the step graph should hold the gradient all-reduce (a
        capturable RCCL process group is up).  With world_size 1 this is the
        in-graph data-parallel form reduced over one rank (tests)."""
        if self.dp_in_graph is False or not (dist.is_available() and dist.is_initialized()):
            return False
        if self.dp_in_graph is None and dist.get_backend() != "nccl":
            return False  # gloo collectives run on the host: not capturable
        return True

    def optimizer_step(self, stepped=False):
        """Gradient exchange, GradScaler + optimizer step, LR schedule.
        stepped: the exchange (if any) and the optimizer already ran inside
        the replayed step graph (native step), only the schedule advances."""
        if not stepped:
            if self.world_size > 1:
                flat_allreduce_(self.model.parameters(), self.world_size)
            if self.native_adam():
                self._native_opt.step()
            else:
                self.scaler.step(self.optimizer)
                self.scaler.update()
        inv = getattr(self.model, "invalidate_infer_operands", None)
        if inv is not None:
            inv()  # the parameters moved in place (eval-frame operand cache)
        if self.scheduler_update_every_step:
            self.lr_scheduler.step()

    def train_iteration(self, data):
        """One optimisation step of the SDS loop (reference utils.py:693-715
        minus the per-step loss.item())."""
        if self.model.cuda_ray and self.global_step % self.opt.update_extra_interval == 0:
            with torch.autocast("cuda", enabled=self.amp, dtype=self.amp_dtype):
                self.model.update_extra_state()
        self.local_step += 1
        self.global_step += 1
        shading, ambient_ratio = self.pick_shading()
        native_only = shading != "albedo" or not self.fused_backward
        if self._graph_eligible(shading) and (not native_only or
                                              ("pose" in data and "intrinsics" in data)):
            return self._graph_iteration(data, shading, ambient_ratio)
        self.optimizer.zero_grad()
        with torch.autocast("cuda", enabled=self.amp, dtype=self.amp_dtype):
            pred_rgbs, pred_ws, loss = self.train_step(data, shading, ambient_ratio)
        self.backward_and_step(loss)
        # detached: a caller holding the loss must not keep this step's autograd
        # graph (and its AccumulateGrad nodes, bound to this stream) alive into
        # a later graph capture on another stream
        return loss.detach() if torch.is_tensor(loss) else loss

    # ------------------------------------------------------------ graph step
    def _graph_eligible(self, shading):
        if not (self.graph_step and self.amp and self.model.cuda_ray
                and hasattr(self.guidance, "sds_grad") and self.device.type == "cuda"):
            return False
        if not self.fused_backward or shading != "albedo" or self.bf16:
            # the two-pass backward and the normal-shaded steps are graphed only
            # as the native step
            from . import native_step as _native
            return self.native_step and _native.eligible(self, shading)
        return (self.graph_step and self.fp16 and self.model.cuda_ray and shading == "albedo"
                and self.fused_backward and hasattr(self.guidance, "sds_grad")
                and self.device.type == "cuda")

    def _bucketed(self, shading):
        """The step runs as BucketedModuleStep: the module path (unfused field)
        where no native step applies."""
        from . import native_step as _native
        if not self.module_buckets or getattr(self.model, "fused_field", True):
            return False
        return not (self.native_step and _native.eligible(self, shading))

    def _graph_iteration(self, data, shading, ambient_ratio):
        """The step as a HIP-graph replay (nerf/graph.py): captured on the first
        eligible step of each (shading, resolution), replayed afterwards."""
        from .graph import BucketedModuleStep, GraphedTrainStep
        model = self.model
        if self._capture_stream is None:
            self._capture_stream = torch.cuda.Stream(device=self.device)
        key = (shading, ambient_ratio, data["H"], data["W"])
        g = self._graphs.get(key)
        if g is None and self._bucketed(shading):
            g = BucketedModuleStep(self, data["H"], data["W"], shading, ambient_ratio,
                                   self._capture_stream)
            self._graphs[key] = g
        if isinstance(g, BucketedModuleStep):
            text_z = self.text_z[data["dir"]] if self.opt.dir_text else self.text_z
            row = model.local_step % 16
            model.local_step += 1
            loss = g.step(data, text_z)
            model.step_counter[row].copy_(g.counter)
            model.last_counter = g.counter
            self.optimizer_step()
            return loss
        # the prompt embedding of the view class: an index op whose CPU index is
        # copied from pageable memory (which waits for the stream); the native
        # step's synthetic guidance does not read it
        text_z = None
        if g is None or g.native is None:
            text_z = self.text_z[data["dir"]] if self.opt.dir_text else self.text_z
        row = model.local_step % 16
        if g is None:
            g = GraphedTrainStep(self, data, shading, ambient_ratio, text_z, self._capture_stream)
            g.capture(data)  # run_cuda advanced model.local_step while recording
            self._graphs[key] = g
        else:
            model.local_step += 1
        g.load(data, text_z)
        if self.step_hook is not None:
            self.step_hook(g)  # bench.py kernel timing: the eager twin of the replay
        else:
            g.replay()
        model.step_counter[row].copy_(g.counter)
        self.optimizer_step(stepped=g.optimizer_in_graph)
        return g.loss

    def train_one_epoch(self, loader):
        self.log(f"==> Start Training {self.workspace} Epoch {self.epoch}, "
                 f"lr={self.optimizer.param_groups[0]['lr']:.6f} ...")
        self.model.train()
        self.local_step = 0
        total = torch.zeros((), device=self.device)
        for data in loader:
            loss = self.train_iteration(data)
            if torch.is_tensor(loss):
                total += loss.detach().float()
        if self.ema is not None:
            self.ema.update()
        average_loss = total.item() / max(1, self.local_step)
        self.stats["loss"].append(average_loss)
        if not self.scheduler_update_every_step:
            self.lr_scheduler.step()
        self.log(f"==> Finished Epoch {self.epoch}. loss={average_loss:.6f}")

    def train(self, train_loader, valid_loader, max_epochs):
        assert self.text_z is not None, "Training must provide a text prompt!"
        start = time.time()
        for epoch in range(self.epoch + 1, max_epochs + 1):
            self.epoch = epoch
            self.train_one_epoch(train_loader)
            if self.workspace is not None and self.local_rank == 0:
                self.save_checkpoint(full=True, best=False)
        self.log(f"[INFO] training takes {(time.time() - start) / 60:.4f} minutes.")

    # ------------------------------------------------------------ eval
    @torch.no_grad()
    def test_step(self, data, bg_color=None, perturb=False):
        rays_o, rays_d = data["rays_o"], data["rays_d"]
        B, N = rays_o.shape[:2]
        H, W = data["H"], data["W"]
        if H * W == N:  # row-major images: the fused renderer's queue takes 8 x 8 tiles
            self.model.infer_tile_w = W
        out = self.model.render(rays_o, rays_d, staged=True, perturb=perturb, light_d=None,
                                ambient_ratio=1.0, shading="albedo", force_all_rays=True,
                                bg_color=bg_color, **vars(self.opt))
        return out["image"].reshape(B, H, W, 3), out["depth"].reshape(B, H, W)

    # ------------------------------------------------------------ checkpoints
    def save_mesh(self, save_path=None, resolution=128):
        """utils.py:459-470: export the density isosurface under
        `workspace/mesh` (NeRFRenderer.export_mesh, nerf/mesh.py)."""
        if save_path is None:
            save_path = os.path.join(self.workspace, "mesh")
        self.log(f"==> Saving mesh to {save_path}")
        os.makedirs(save_path, exist_ok=True)
        self.model.export_mesh(save_path, resolution=resolution)
        self.log("==> Finished saving mesh.")

    def save_checkpoint(self, name=None, full=False, best=False):
        """Same checkpoint dict layout as the reference (utils.py:847-902)."""
        if name is None:
            name = f"{self.name}_ep{self.epoch:04d}"
        state = {"epoch": self.epoch, "global_step": self.global_step, "stats": self.stats}
        if self.model.cuda_ray:
            state["mean_count"] = self.model.mean_count
            state["mean_density"] = self.model.mean_density
        if full:
            state["optimizer"] = self.optimizer.state_dict()
            state["lr_scheduler"] = self.lr_scheduler.state_dict()
            state["scaler"] = self.scaler.state_dict()
            if self.ema is not None:
                state["ema"] = self.ema.state_dict()
        state["model"] = self.model.state_dict()
        if not best:
            path = f"{name}.pth"
            self.stats["checkpoints"].append(path)
            if len(self.stats["checkpoints"]) > self.max_keep_ckpt:
                old = os.path.join(self.ckpt_path, self.stats["checkpoints"].pop(0))
                if os.path.exists(old):
                    os.remove(old)
            torch.save(state, os.path.join(self.ckpt_path, path))
        else:
            torch.save(state, self.best_path)

    def load_checkpoint(self, checkpoint=None, model_only=False):
        if checkpoint is None:
            found = sorted(glob.glob(f"{self.ckpt_path}/{self.name}_ep*.pth"))
            if not found:
                self.log("[WARN] No checkpoint found, model randomly initialized.")
                return
            checkpoint = found[-1]
        # our own checkpoints only: tensors + plain containers
        ckpt = torch.load(checkpoint, map_location=self.device, weights_only=True)
        if "model" not in ckpt:
            self.model.load_state_dict(ckpt)
            return
        missing, unexpected = self.model.load_state_dict(ckpt["model"], strict=False)
        if len(missing) > 0:
            self.log(f"[WARN] missing keys: {missing}")
        if len(unexpected) > 0:
            self.log(f"[WARN] unexpected keys: {unexpected}")
        if self.model.cuda_ray:
            self.model.mean_count = ckpt.get("mean_count", self.model.mean_count)
            self.model.mean_density = ckpt.get("mean_density", self.model.mean_density)
        if hasattr(self.model, "invalidate_infer_operands"):
            self.model.invalidate_infer_operands()
        if model_only:
            return
        self.stats = ckpt.get("stats", self.stats)
        self.epoch = ckpt.get("epoch", 0)
        self.global_step = ckpt.get("global_step", 0)
        for key, obj in (("optimizer", self.optimizer), ("lr_scheduler", self.lr_scheduler),
                         ("scaler", self.scaler)):
            if key in ckpt:
                try:
                    obj.load_state_dict(ckpt[key])
                except Exception:  # noqa: BLE001 - mismatched groups: keep fresh state
                    self.log(f"[WARN] failed to load {key}.")
        if self.ema is not None and "ema" in ckpt:
            self.ema.load_state_dict(ckpt["ema"])
        # captured step graphs hold the old optimizer-state pointers
        self._graphs = {}
        self._native_opt = None
