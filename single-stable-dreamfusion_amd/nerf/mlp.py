"""Tiny-MLP forward/backward with a split-K weight gradient.

The reference's MLP is a stack of nn.Linear under autocast (network_grid.py:
13-32).  On ROCm the backward of nn.Linear forms each weight gradient as ONE
GEMM  dW = dY^T X  with K = number of samples (~770k at 128x128) and a
64x32 / 64x64 / 4x64 output: hipBLASLt picks a single tile column for it and
the three dW GEMMs took 7.7 ms of a 21.6 ms step on MI355X.  Here the samples
are cut into S chunks and the partial products are formed by one batched GEMM
(S independent tiles -> all CUs busy), then summed in f32.

Numerics follow autocast: fp16 GEMMs with f32 accumulation, fp16 activations,
f32 weight gradients (as autocast's cast-op backward delivers them).
"""
import torch
import torch.nn.functional as F
from torch.autograd import Function
from torch.amp import custom_bwd, custom_fwd

_CHUNK = 4096  # rows per split-K chunk
_SPLIT_MIN = 2 * _CHUNK  # split only when K (rows) is larger than this


_BMM_F32_OUT = [True]


def _bmm_f32(a, b):
    """Batched GEMM with f32 output (f16 inputs keep f32 partial sums)."""
    if _BMM_F32_OUT[0] and a.dtype == torch.float16:
        try:
            return torch.bmm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            _BMM_F32_OUT[0] = False
    return torch.bmm(a, b).float()


def _split_k_wgrad(dy, x):
    """sum over rows of dy^T x, i.e. [N, K] = dy[M, N]^T @ x[M, K], in f32."""
    m = dy.shape[0]
    if m <= _SPLIT_MIN:
        # small K (e.g. the per-ray background MLP): one GEMM is fine
        return (dy.t() @ x).float()
    s = m // _CHUNK
    head = s * _CHUNK
    dyc = dy[:head].view(s, _CHUNK, -1)
    xc = x[:head].view(s, _CHUNK, -1)
    out = _bmm_f32(dyc.transpose(1, 2), xc).sum(0)
    if head < m:
        out += (dy[head:].t() @ x[head:]).float()
    return out


class _MLPFunction(Function):
    @staticmethod
    @custom_fwd(device_type="cuda")
    def forward(ctx, x, *params):
        """params = (w0, b0, w1, b1, ..., w_{n-1}, b_{n-1}) (nn.Linear layout).
        ReLU between layers, none after the last."""
        half = torch.is_autocast_enabled("cuda")
        dt = torch.float16 if half else x.dtype
        n = len(params) // 2
        h = x.to(dt)
        acts = [h]
        ws = []
        for i in range(n):
            w = params[2 * i].to(dt)
            b = params[2 * i + 1].to(dt)
            ws.append(w)
            h = F.linear(h, w, b)
            if i != n - 1:
                h = torch.relu_(h)
            acts.append(h)
        ctx.save_for_backward(*acts[:-1], *ws)
        ctx.n = n
        ctx.in_dtype = x.dtype
        ctx.param_dtypes = [p.dtype for p in params]
        return h

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, g):
        n = ctx.n
        saved = ctx.saved_tensors
        acts, ws = saved[:n], saved[n:]
        grads = [None] * (2 * n)
        dy = g.to(acts[0].dtype).contiguous()
        for i in reversed(range(n)):
            if i != n - 1:
                dy = dy * (acts[i + 1] > 0)  # ReLU of layer i's output
            x = acts[i]
            grads[2 * i] = _split_k_wgrad(dy, x).to(ctx.param_dtypes[2 * i])
            grads[2 * i + 1] = torch.sum(dy, 0, dtype=torch.float32).to(ctx.param_dtypes[2 * i + 1])
            if i > 0 or ctx.needs_input_grad[0]:
                dy = dy @ ws[i]
        dx = dy.to(ctx.in_dtype) if ctx.needs_input_grad[0] else None
        return (dx, *grads)


def mlp_forward(x, layers):
    """Run a list of nn.Linear layers (ReLU between) through _MLPFunction."""
    params = []
    for lin in layers:
        params += [lin.weight, lin.bias]
    return _MLPFunction.apply(x, *params)
