"""Grid-backbone NeRF field (behavioural mirror of reference nerf/network_grid.py).

Tiled multi-resolution grid (16 levels x 2 channels, 2^16 rows per level,
resolution 16 -> 2048*bound) + ReLU MLP 32 -> 64 -> 64 -> 4, a Gaussian density
blob at the origin, finite-difference normals and a frequency-encoded
background MLP 39 -> 64 -> 3.  Module names, parameter shapes and creation
order (hence seeded initialisation and state_dict keys) match the reference
(network_grid.py:35-181).  Its forward goes through the same reference-API
modules (GridEncoder, FreqEncoder, trunc_exp, raymarching.*) that the
reference file calls; with `fused_field = False` (and the Trainer's
`native_step = False`) they run one by one as separate autograd nodes — the
path the reference file takes on this package — and bench.py times that path
as `module_path`.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

import raymarching
from activation import trunc_exp
from encoding import get_encoder

from . import field as _field
from .mlp import mlp_forward
from .renderer import NeRFRenderer
from .utils import safe_normalize


class MLP(nn.Module):
    """Bias-ful Linear stack with in-place ReLU between layers (network_grid.py:13-32)."""

    def __init__(self, dim_in, dim_out, dim_hidden, num_layers, bias=True):
        super().__init__()
        self.dim_in, self.dim_out = dim_in, dim_out
        self.dim_hidden, self.num_layers = dim_hidden, num_layers
        widths = [dim_in] + [dim_hidden] * (num_layers - 1) + [dim_out]
        self.net = nn.ModuleList(nn.Linear(widths[i], widths[i + 1], bias=bias)
                                 for i in range(num_layers))

    def forward(self, x):
        if x.is_cuda:
            # same math as the Linear/ReLU stack, split-K weight gradients (mlp.py)
            return mlp_forward(x, self.net)
        last = self.num_layers - 1
        for i, layer in enumerate(self.net):
            x = layer(x)
            if i != last:
                x = F.relu(x, inplace=True)
        return x


# unit offsets of the central-difference stencil (+x, -x, +y, -y, +z, -z)
_STENCIL = ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1))


class NeRFNetwork(NeRFRenderer):
    def __init__(self, opt, num_layers=3, hidden_dim=64, num_layers_bg=2, hidden_dim_bg=64):
        super().__init__(opt)
        self.num_layers = num_layers
        self.hidden_dim = hidden_dim
        self.encoder, self.in_dim = get_encoder("tiledgrid", input_dim=3, log2_hashmap_size=16,
                                                desired_resolution=2048 * self.bound)
        self.sigma_net = MLP(self.in_dim, 4, hidden_dim, num_layers, bias=True)
        # encoder + MLP + heads as one native node (nerf/field.py) where it
        # applies; False: GridEncoder -> MLP -> trunc_exp / sigmoid one by one
        self.fused_field = True
        if self.bg_radius > 0:
            self.num_layers_bg = num_layers_bg
            self.hidden_dim_bg = hidden_dim_bg
            self.encoder_bg, self.in_dim_bg = get_encoder("frequency", input_dim=3)
            self.bg_net = MLP(self.in_dim_bg, 3, hidden_dim_bg, num_layers_bg, bias=True)
        else:
            self.bg_net = None

    def gaussian(self, x):
        """Density blob at the scene centre: 5 * exp(-|x|^2 / (2 * 0.2^2))."""
        return 5 * torch.exp(-(x ** 2).sum(-1) / (2 * 0.2 ** 2))

    def common_forward(self, x):
        """x [N, 3] in [-bound, bound] -> sigma [N] (f32), albedo [N, 3]."""
        if self.fused_field and _field.eligible(self.encoder, self.sigma_net.net, x):
            # encoder + MLP + heads as one native node (nerf/field.py)
            # capacity-sized samples of the device-count march carry their live count
            return _field.grid_field(x, self.bound, self.encoder, self.sigma_net.net,
                                     m_dev=raymarching.live_rows(x))
        h = self.sigma_net(self.encoder(x, bound=self.bound))
        sigma = trunc_exp(h[..., 0] + self.gaussian(x))
        albedo = torch.sigmoid(h[..., 1:])
        return sigma, albedo

    def finite_difference_normal(self, x, epsilon=1e-2):
        vals = []
        for off in _STENCIL:
            shift = torch.tensor([off], dtype=x.dtype, device=x.device) * epsilon
            sigma, _ = self.common_forward((x + shift).clamp(-self.bound, self.bound))
            vals.append(sigma)
        grad = torch.stack([0.5 * (vals[2 * i] - vals[2 * i + 1]) / epsilon for i in range(3)],
                           dim=-1)
        return -grad

    def normal(self, x):
        n = safe_normalize(self.finite_difference_normal(x))
        n[torch.isnan(n)] = 0
        return n

    def forward(self, x, d, l=None, ratio=1, shading="albedo"):
        """x, d: [N, 3]; l: [3] light direction; ratio: ambient share.
        Returns sigma [N], color [N, 3], normal [N, 3] or None."""
        if shading == "albedo":
            sigma, color = self.common_forward(x)
            return sigma, color, None
        sigma, albedo = self.common_forward(x)
        normal = self.normal(x)
        lambertian = ratio + (1 - ratio) * (normal @ l).clamp(min=0)
        if shading == "textureless":
            color = lambertian.unsqueeze(-1).repeat(1, 3)
        elif shading == "normal":
            color = (normal + 1) / 2
        else:  # lambertian
            color = albedo * lambertian.unsqueeze(-1)
        return sigma, color, normal

    def density(self, x):
        sigma, albedo = self.common_forward(x)
        return {"sigma": sigma, "albedo": albedo}

    def native_infer_field(self, shading, x):
        if shading != "albedo" or not self.fused_field:
            return None
        if not _field.eligible(self.encoder, self.sigma_net.net, x):
            return None
        return self.encoder, list(self.sigma_net.net)

    def native_background_layers(self):
        from freqencoder import FreqEncoder
        if self.bg_radius <= 0 or not isinstance(self.encoder_bg, FreqEncoder):
            return None
        if self.encoder_bg.input_dim != 3 or self.encoder_bg.degree != 6:
            return None
        layers = list(self.bg_net.net)
        return layers if len(layers) == 2 else None

    def background(self, d):
        return torch.sigmoid(self.bg_net(self.encoder_bg(d)))

    def get_params(self, lr):
        groups = [{"params": self.encoder.parameters(), "lr": lr * 10},
                  {"params": self.sigma_net.parameters(), "lr": lr}]
        if self.bg_radius > 0:
            groups.append({"params": self.encoder_bg.parameters(), "lr": lr * 10})
            groups.append({"params": self.bg_net.parameters(), "lr": lr})
        return groups
