"""trunc_exp (mirror of reference activation.py:5-18): exp in f32 forward,
gradient g * exp(clamp(x, -15, 15))."""
import torch
from torch.autograd import Function
from torch.amp import custom_bwd, custom_fwd


class _trunc_exp(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float)
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.exp(x.clamp(-15, 15))


trunc_exp = _trunc_exp.apply
