"""Spherical-harmonics encoder (mirror of reference shencoder/sphere_harmonics.py):
real SH of degree 1..8 (degree^2 outputs) of 3-D directions."""
import torch
import torch.nn as nn
from torch.autograd import Function
from torch.amp import custom_bwd, custom_fwd

import _shencoder as _backend


class _sh_encoder(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, inputs, degree, calc_grad_inputs=False):
        """inputs [B, 3] -> [B, degree^2]; dy_dx [B, 3*degree^2] kept for backward."""
        inputs = inputs.contiguous()
        B, D = inputs.shape
        out_dim = degree ** 2
        outputs = torch.empty(B, out_dim, dtype=inputs.dtype, device=inputs.device)
        dy_dx = (torch.empty(B, D * out_dim, dtype=inputs.dtype, device=inputs.device)
                 if calc_grad_inputs else None)
        _backend.sh_encode_forward(inputs, outputs, B, D, degree, dy_dx)
        ctx.save_for_backward(inputs, dy_dx)
        ctx.dims = (B, D, degree)
        return outputs

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad):
        inputs, dy_dx = ctx.saved_tensors
        if dy_dx is None:
            return None, None, None
        B, D, degree = ctx.dims
        grad_inputs = torch.zeros_like(inputs)
        _backend.sh_encode_backward(grad.contiguous(), inputs, B, D, degree, dy_dx, grad_inputs)
        return grad_inputs, None, None


sh_encode = _sh_encoder.apply


class SHEncoder(nn.Module):
    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        self.input_dim = input_dim
        self.degree = degree
        self.output_dim = degree ** 2
        assert self.input_dim == 3, "SH encoder only support input dim == 3"
        assert 0 < self.degree <= 8, "SH encoder only supports degree in [1, 8]"

    def __repr__(self):
        return f"SHEncoder: input_dim={self.input_dim} degree={self.degree}"

    def forward(self, inputs, size=1):
        x = inputs / size
        lead = list(x.shape[:-1])
        out = sh_encode(x.reshape(-1, self.input_dim), self.degree, x.requires_grad)
        return out.reshape(lead + [self.output_dim])
