"""Score-distillation guidance (reference nerf/sd.py) on PyTorch-ROCm.

`StableDiffusion` keeps the reference's interface (get_text_embeds,
train_step -> 0 after an injected latent backward, sd.py:54-118) and adds
`sds_grad`, which returns (latents, grad) so the trainer can fuse the latent
backward with the regulariser backward.  The real model needs `diffusers` and
LOCAL weights (nothing is ever fetched by name).

`InjectedSDS` is the benchmark's offline guidance (a seeded w(t)-weighted N(0,1)
gradient injected at pred_rgb).  `SyntheticSDS` is the
fuller offline stand-in: the same
SDS arithmetic (timestep draw, scaled_linear alphas_cumprod, add_noise,
classifier-free guidance with scale 100, w(t) = 1 - alphas_cumprod[t],
gradient injection at the latents) around fixed random 1x1-conv "VAE" /
"UNet" maps instead of SD's networks, so the render graph sees the same
backward topology (bilinear 512^2 upsample -> encoder -> latents).
"""
import os
import zlib

import torch
import torch.nn as nn
import torch.nn.functional as F


def scaled_linear_alphas_cumprod(n=1000, beta_start=0.00085, beta_end=0.012):
    """alphas_cumprod of diffusers' 'scaled_linear' schedule (sd.py:49-50)."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


def add_noise(alphas_cumprod, latents, noise, t):
    """DDPM forward process x_t = sqrt(a_t) x_0 + sqrt(1 - a_t) eps."""
    a = alphas_cumprod[t].to(latents.dtype).flatten()
    while a.dim() < latents.dim():
        a = a.unsqueeze(-1)
    return a.sqrt() * latents + (1 - a).sqrt() * noise


def cfg_combine(noise_pred, guidance_scale):
    uncond, text = noise_pred.chunk(2)
    return uncond + guidance_scale * (text - uncond)


def seeded_text_embeds(prompt, negative_prompt, dim, device):
    """Offline stand-in for CLIP text embeddings: [negatives..., prompts...]
    each a [77, dim] N(0, 1) tensor seeded by the text's CRC32."""
    out = []
    for text in list(negative_prompt) + list(prompt):
        gen = torch.Generator().manual_seed(zlib.crc32(text.encode("utf-8")))
        out.append(torch.randn(77, dim, generator=gen))
    return torch.stack(out).to(device)


class _SDSBase(nn.Module):
    num_train_timesteps = 1000

    def __init__(self, device):
        super().__init__()
        self.device = device
        self.min_step = int(self.num_train_timesteps * 0.02)
        self.max_step = int(self.num_train_timesteps * 0.98)
        self.register_buffer("alphas", scaled_linear_alphas_cumprod(self.num_train_timesteps))

    # subclass hooks
    def encode_imgs(self, imgs):
        raise NotImplementedError

    def predict_noise(self, latent_model_input, t, text_embeddings):
        raise NotImplementedError

    def sds_grad(self, text_embeddings, pred_rgb, guidance_scale=100):
        """Returns (latents, grad): the SDS gradient w(t) (eps_hat - eps) to be
        injected at the latents (sd.py:74-115 without the backward call)."""
        pred_rgb_512 = F.interpolate(pred_rgb, (512, 512), mode="bilinear", align_corners=False)
        t = torch.randint(self.min_step, self.max_step + 1, [1], dtype=torch.long,
                          device=pred_rgb.device)
        latents = self.encode_imgs(pred_rgb_512)
        with torch.no_grad():
            noise = torch.randn_like(latents)
            latents_noisy = add_noise(self.alphas, latents, noise, t)
            noise_pred = self.predict_noise(torch.cat([latents_noisy] * 2), t, text_embeddings)
        noise_pred = cfg_combine(noise_pred, guidance_scale)
        w = 1 - self.alphas[t]
        return latents, w * (noise_pred - noise)

    def train_step(self, text_embeddings, pred_rgb, guidance_scale=100):
        latents, grad = self.sds_grad(text_embeddings, pred_rgb, guidance_scale)
        latents.backward(gradient=grad, retain_graph=True)
        return 0  # dummy loss value, as the reference


class SyntheticSDS(_SDSBase):
    """Offline SDS stand-in (see module docstring).  Deterministic given the
    torch seed; text embeddings are seeded random [2, 77, dim] tensors."""

    def __init__(self, device, text_dim=768, seed=1234):
        super().__init__(device)
        g = torch.Generator().manual_seed(seed)
        self.text_dim = text_dim
        # "VAE encoder": 8x8 average pool + 1x1 conv 3 -> 4, scaled by 0.18215
        self.enc_w = nn.Parameter(torch.randn(4, 3, 1, 1, generator=g) * 0.5, requires_grad=False)
        # "UNet": 1x1 conv 4 -> 4 on the noisy latents + a text-dependent bias
        self.eps_w = nn.Parameter(torch.randn(4, 4, 1, 1, generator=g) * 0.1, requires_grad=False)
        self.txt_w = nn.Parameter(torch.randn(4, text_dim, generator=g) * 0.01, requires_grad=False)
        self.to(device)

    def get_text_embeds(self, prompt, negative_prompt):
        return seeded_text_embeds(prompt, negative_prompt, self.text_dim, self.device)

    def encode_imgs(self, imgs):
        x = F.avg_pool2d(2 * imgs - 1, 8)
        return F.conv2d(x, self.enc_w.to(x.dtype)) * 0.18215

    def predict_noise(self, latent_model_input, t, text_embeddings):
        eps = F.conv2d(latent_model_input, self.eps_w.to(latent_model_input.dtype))
        bias = text_embeddings.mean(1).to(eps.dtype) @ self.txt_w.t().to(eps.dtype)  # [2, 4]
        return eps + bias[:, :, None, None]


class InjectedSDS(_SDSBase):
    """The benchmark's guidance (SURVEY.md §8(d) "synthetic SDS"): SD's VAE /
    UNet are absent offline, so the SDS gradient w(t) (eps_hat - eps) is
    replaced by a seeded N(0, 1) gradient of pred_rgb's shape, weighted by
    w(t) = 1 - alphas_cumprod[t] of a drawn timestep, and injected at pred_rgb
    (the backward topology of the render graph minus VAE / UNet).  The full
    SDS arithmetic around stand-in networks is `SyntheticSDS`."""

    def __init__(self, device, text_dim=768):
        super().__init__(device)
        self.text_dim = text_dim
        self.to(device)

    def get_text_embeds(self, prompt, negative_prompt):
        return seeded_text_embeds(prompt, negative_prompt, self.text_dim, self.device)

    def sds_grad(self, text_embeddings, pred_rgb, guidance_scale=100):
        t = torch.randint(self.min_step, self.max_step + 1, [1], dtype=torch.long,
                          device=pred_rgb.device)
        w = 1 - self.alphas[t]
        return pred_rgb, w * torch.randn_like(pred_rgb, dtype=torch.float32)


class StableDiffusion(_SDSBase):
    """Real SD-1.5 / SD-2.1-base guidance from a LOCAL diffusers checkpoint
    directory (env DFHIP_SD_PATH or `model_path`).  Requires `diffusers` and
    `transformers`; never downloads."""

    def __init__(self, device, model_path=None, dtype=torch.float16):
        super().__init__(device)
        model_path = model_path or os.environ.get("DFHIP_SD_PATH")
        if not model_path or not os.path.isdir(model_path):
            raise RuntimeError("StableDiffusion needs a local diffusers checkpoint directory "
                               "(set DFHIP_SD_PATH); use SyntheticSDS offline")
        from diffusers import AutoencoderKL, UNet2DConditionModel  # noqa: import-outside-toplevel
        from transformers import CLIPTextModel, CLIPTokenizer  # noqa: import-outside-toplevel
        kw = dict(local_files_only=True, torch_dtype=dtype)
        self.vae = AutoencoderKL.from_pretrained(model_path, subfolder="vae", **kw).to(device)
        self.tokenizer = CLIPTokenizer.from_pretrained(model_path, subfolder="tokenizer",
                                                       local_files_only=True)
        self.text_encoder = CLIPTextModel.from_pretrained(model_path, subfolder="text_encoder",
                                                          **kw).to(device)
        self.unet = UNet2DConditionModel.from_pretrained(model_path, subfolder="unet",
                                                         **kw).to(device)

    def get_text_embeds(self, prompt, negative_prompt):
        def enc(texts):
            ids = self.tokenizer(texts, padding="max_length", truncation=True,
                                 max_length=self.tokenizer.model_max_length,
                                 return_tensors="pt").input_ids.to(self.device)
            with torch.no_grad():
                return self.text_encoder(ids)[0]
        return torch.cat([enc(negative_prompt), enc(prompt)])

    def encode_imgs(self, imgs):
        post = self.vae.encode(2 * imgs - 1).latent_dist
        return post.sample() * 0.18215

    def predict_noise(self, latent_model_input, t, text_embeddings):
        return self.unet(latent_model_input, t, encoder_hidden_states=text_embeddings).sample
