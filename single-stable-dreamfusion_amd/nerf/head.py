"""Native per-ray tail of the render and the entropy regulariser (csrc/head.hip).

`ray_head` replaces the end of NeRFRenderer.run_cuda (reference
nerf/renderer.py:536-551): background network (network_grid.py:158-167),
`image + (1 - ws) * bg`, the depth normalisation and the mask, with pred_rgb
written channel-major so the train step's reshape/permute/contiguous
(utils.py:369) is a view.  `ray_entropy` is the `lambda_entropy` term of
Trainer.train_step (utils.py:386-391).  Both are autograd Functions with
native forward and backward; they apply only on the GPU with the reference's
shapes (background MLP 39 -> 64 -> 3, one batch of rays), everything else
keeps the torch expressions.
"""
import torch
from torch.autograd import Function

import _dfhip
from _dfhip import ptr


def _f32c(t):
    return t.detach().float().contiguous()


class _RayHead(Function):
    @staticmethod
    def forward(ctx, ws, depth, image, rays_d, nears, fars, bg_color, w1, b1, w2, b2):
        N = ws.numel()
        dev = ws.device
        ws_, depth_, image_ = _f32c(ws), _f32c(depth), _f32c(image)
        nears_, fars_ = _f32c(nears), _f32c(fars)
        net = w1 is not None
        rays_d_ = _f32c(rays_d) if net else None
        bg_ = _f32c(bg_color) if (bg_color is not None and not net) else None
        wts = [_f32c(w) for w in (w1, b1, w2, b2)] if net else [None] * 4
        out_image = torch.empty(3, N, device=dev)
        out_depth = torch.empty(N, device=dev)
        mask = torch.empty(N, dtype=torch.bool, device=dev)  # written as 0 / 1 bytes
        _dfhip.call("dfhip_ray_head_forward", N, ptr(ws_), ptr(depth_), ptr(image_),
                    ptr(rays_d_), ptr(nears_), ptr(fars_), *[ptr(w) for w in wts], ptr(bg_),
                    ptr(out_image), ptr(out_depth), ptr(mask), _dfhip.stream())
        ctx.save_for_backward(ws_, rays_d_, bg_, *wts)
        ctx.net = net
        ctx.bg_grad = bg_color is not None and not net and bg_color.requires_grad
        ctx.mark_non_differentiable(mask)
        return out_image, out_depth, mask

    @staticmethod
    def backward(ctx, g_image, g_depth, g_mask):
        # depth carries no gradient on this path: the compositing backward
        # ignores it (reference raymarching.py:275)
        ws, rays_d, bg, w1, b1, w2, b2 = ctx.saved_tensors
        N = ws.numel()
        dev = ws.device
        if g_image is None:
            g_image = torch.zeros(3, N, device=dev)
        g_image = g_image.float().contiguous()
        grad_image = torch.empty(N, 3, device=dev)
        grad_ws = torch.empty(N, device=dev)
        grad_bg = torch.empty(N, 3, device=dev) if ctx.bg_grad else None
        grads = [None] * 4
        partial = None
        if ctx.net:
            grads = [torch.empty_like(w) for w in (w1, b1, w2, b2)]
            partial = torch.empty(int(_dfhip.load().dfhip_ray_head_partial_floats(N)),
                                  device=dev)
        _dfhip.call("dfhip_ray_head_backward", N, ptr(g_image), ptr(ws), ptr(rays_d),
                    ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(bg), ptr(grad_image), ptr(grad_ws),
                    ptr(grad_bg), ptr(partial), *[ptr(g) for g in grads], _dfhip.stream())
        return (grad_ws, None, grad_image, None, None, None, grad_bg, *grads)


def ray_head(ws, depth, image, rays_d, nears, fars, bg_color=None, bg_layers=None):
    """ws [N], depth [N] (relative, as composited), image [N, 3] -> (image_chw
    [3, N], depth [N] normalised, mask [N] bool).  bg_layers: the background
    MLP's two nn.Linear (39 -> 64 -> 3), or None to mix `bg_color` ([N, 3] or
    None for white)."""
    if bg_layers is not None:
        l1, l2 = bg_layers
        return _RayHead.apply(ws, depth, image, rays_d, nears, fars, None, l1.weight, l1.bias,
                              l2.weight, l2.bias)
    return _RayHead.apply(ws, depth, image, rays_d, nears, fars, bg_color, None, None, None,
                          None)


def head_eligible(ws, bg_layers):
    if not ws.is_cuda:
        return False
    if bg_layers is None:
        return True
    if len(bg_layers) != 2:
        return False
    l1, l2 = bg_layers
    return (tuple(l1.weight.shape) == (64, 39) and tuple(l2.weight.shape) == (3, 64)
            and l1.bias is not None and l2.bias is not None)


class _RayEntropy(Function):
    @staticmethod
    def forward(ctx, ws, lam):
        ws_ = _f32c(ws)
        loss = torch.empty((), device=ws.device)
        _dfhip.call("dfhip_entropy_forward", ws_.numel(), ptr(ws_), float(lam), ptr(loss),
                    _dfhip.stream())
        ctx.save_for_backward(ws_)
        ctx.lam = float(lam)
        ctx.shape = ws.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        (ws,) = ctx.saved_tensors
        grad = torch.empty_like(ws)
        g = g.float().contiguous()
        _dfhip.call("dfhip_entropy_backward", ws.numel(), ptr(ws), ptr(g), ctx.lam, ptr(grad),
                    _dfhip.stream())
        return grad.view(ctx.shape), None


def ray_entropy(ws, lam):
    """lam * mean(-a log2 a - (1 - a) log2(1 - a)), a = clamp(ws, 1e-5, 1 - 1e-5)
    (reference utils.py:386-391), as a scalar f32 tensor."""
    return _RayEntropy.apply(ws, lam)
