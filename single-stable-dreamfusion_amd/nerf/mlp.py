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

For the reference's sigma_net shape (32 -> 64 -> 64 -> 4 with biases) under
fp16 / bf16 autocast on the GPU the whole stack is ONE MFMA kernel each way
(csrc/fieldmlp.hip dfhip_mlp_forward / dfhip_mlp_backward: the hidden
activations never reach HBM, the backward recomputes them, the weight
gradients are deterministic per-workgroup partials): the torch form above
took ~0.9 ms of GEMMs, ReLU masks and bias reductions per 128 x 128 step
(rocprofv3, gpurun_out/mp0).  Capacity-sized inputs carrying a device
live-row count (raymarching.live_rows) are processed up to that count.
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


_NATIVE_SHAPES = [(64, 32), (64,), (64, 64), (64,), (4, 64), (4,)]


def _native_dtype(x, params):
    """The autocast element type when the MLP kernels take this call, else None."""
    if not (x.is_cuda and x.dim() == 2 and x.shape[1] == 32
            and torch.is_autocast_enabled("cuda")):
        return None
    dt = torch.get_autocast_dtype("cuda")
    if dt not in (torch.float16, torch.bfloat16):
        return None
    if [tuple(p.shape) for p in params] != _NATIVE_SHAPES:
        return None
    if not all(p.is_cuda and p.dtype == torch.float32 for p in params):
        return None
    return dt


class _NativeMLPFunction(Function):
    @staticmethod
    def forward(ctx, x, m_dev, elem, *params):
        """x [cap, 32] -> h [cap, 4] in elem (fp16 / bf16 autocast numerics)."""
        import _fieldmlp
        xe = x.to(elem).contiguous()
        out = torch.empty(xe.shape[0], 4, dtype=elem, device=xe.device)
        _fieldmlp.mlp_forward(xe, [p.detach() for p in params], out, m_dev)
        ctx.save_for_backward(xe, *params)
        ctx.m_dev, ctx.in_dtype = m_dev, x.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        import _fieldmlp
        xe, *params = ctx.saved_tensors
        cap = xe.shape[0]
        dh = g.to(xe.dtype).contiguous()
        dx = torch.empty(cap, 32, dtype=xe.dtype, device=xe.device)
        grads = [torch.empty_like(p) for p in params]
        partial = torch.empty(max(1, _fieldmlp.backward_parts(cap)) * _fieldmlp.params_count(),
                              dtype=torch.float32, device=xe.device)
        _fieldmlp.mlp_backward(xe, [p.detach() for p in params], dh, dx, partial, grads,
                               ctx.m_dev)
        dx = dx.to(ctx.in_dtype) if ctx.needs_input_grad[0] else None
        return (dx, None, None, *grads)


def mlp_forward(x, layers):
    """Run a list of nn.Linear layers (ReLU between): one MFMA kernel each way
    for the reference's sigma_net shape under autocast, _MLPFunction else."""
    params = []
    for lin in layers:
        params += [lin.weight, lin.bias]
    elem = _native_dtype(x, params)
    if elem is not None:
        # capacity-sized rows of the device-count march carry their live count
        m_dev = getattr(x, "_dfhip_live_rows", None)
        return _NativeMLPFunction.apply(x, m_dev, elem, *params)
    return _MLPFunction.apply(x, *params)
