"""Host-side diffusion utilities mirroring ldm/modules/diffusionmodules/util.py.

Schedules are computed once on the host (numpy float64, as the reference does);
the per-step device math (timestep embedding, q_sample, DDIM update) runs in HIP
kernels (encdiff_amd/csrc/elementwise.hip).
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch import nn


def make_beta_schedule(schedule, n_timestep, linear_start=1e-4, linear_end=2e-2, cosine_s=8e-3):
    """util.py:21-70 ('linear' is the one EncDiff configs use)."""
    if schedule == "linear":
        return np.linspace(linear_start ** 0.5, linear_end ** 0.5, n_timestep, dtype=np.float64) ** 2
    if schedule == "cosine":
        ts = np.arange(n_timestep + 1, dtype=np.float64) / n_timestep + cosine_s
        al = np.cos(ts / (1 + cosine_s) * np.pi / 2) ** 2
        al = al / al[0]
        return np.clip(1 - al[1:] / al[:-1], 0, 0.999)
    if schedule == "sqrt_linear":
        return np.linspace(linear_start, linear_end, n_timestep, dtype=np.float64)
    if schedule == "sqrt":
        return np.linspace(linear_start, linear_end, n_timestep, dtype=np.float64) ** 0.5
    raise ValueError(f"schedule '{schedule}' unknown.")


def make_ddim_timesteps(ddim_discr_method, num_ddim_timesteps, num_ddpm_timesteps, verbose=True):
    """util.py:73-87: uniform (or quad) subsequence, shifted by +1."""
    if ddim_discr_method == "uniform":
        c = num_ddpm_timesteps // num_ddim_timesteps
        steps = np.asarray(list(range(0, num_ddpm_timesteps, c)))
    elif ddim_discr_method == "quad":
        steps = ((np.linspace(0, np.sqrt(num_ddpm_timesteps * .8), num_ddim_timesteps)) ** 2).astype(int)
    else:
        raise NotImplementedError(ddim_discr_method)
    out = steps + 1
    if verbose:
        print(f"Selected timesteps for ddim sampler: {out}")
    return out


def make_ddim_sampling_parameters(alphacums, ddim_timesteps, eta, verbose=True):
    """util.py:90-102 (alphacums is the fp32 alphas_cumprod buffer, as in ddim.py:43-45;
    the mixed torch/numpy expression is kept so sigma matches bit for bit)."""
    alphas = alphacums[ddim_timesteps]
    alphas_prev = np.asarray([alphacums[0]] + alphacums[ddim_timesteps[:-1]].tolist())
    sigmas = eta * np.sqrt((1 - alphas_prev) / (1 - alphas) * (1 - alphas / alphas_prev))
    to64 = lambda a: np.asarray(a.numpy() if isinstance(a, torch.Tensor) else a, dtype=np.float64)
    alphas_next = np.asarray(alphacums[ddim_timesteps[1:]].tolist() + [float(alphacums[-1])])
    if verbose:
        print(f"Selected alphas for ddim sampler: a_t: {alphas}; a_(t-1): {alphas_prev}")
    return to64(sigmas), to64(alphas), to64(alphas_prev), to64(alphas_next)


def extract_into_tensor(a, t, x_shape):
    """util.py:124-127."""
    b = t.shape[0]
    return a.gather(-1, t).reshape(b, *((1,) * (len(x_shape) - 1)))


def timestep_embedding(timesteps, dim, max_period=10000, repeat_only=False):
    """util.py:179-199 (host reference form; the UNet computes it in a HIP kernel)."""
    if repeat_only:
        return timesteps[:, None].expand(-1, dim)
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half).to(timesteps.device)
    args = timesteps[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def noise_like(shape, device, repeat=False):
    """util.py:292-295."""
    if repeat:
        return torch.randn((1, *shape[1:]), device=device).repeat(shape[0], *((1,) * (len(shape) - 1)))
    return torch.randn(shape, device=device)


def zero_module(module):
    for p in module.parameters():
        p.detach().zero_()
    return module


class GroupNorm32(nn.GroupNorm):
    """util.py:242-244 (parameter container; compute runs in the HIP GroupNorm kernel)."""

    def forward(self, x):
        return super().forward(x.float()).type(x.dtype)


def normalization(channels):
    return GroupNorm32(32, channels)


def conv_nd(dims, *args, **kwargs):
    if dims == 2:
        return nn.Conv2d(*args, **kwargs)
    if dims == 1:
        return nn.Conv1d(*args, **kwargs)
    return nn.Conv3d(*args, **kwargs)


def linear(*args, **kwargs):
    return nn.Linear(*args, **kwargs)


def mean_flat(tensor):
    return tensor.mean(dim=list(range(1, len(tensor.shape))))
