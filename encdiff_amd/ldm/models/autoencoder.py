"""Frozen VQ first stage -- called as-is (plain PyTorch).

Mirrors ldm/models/autoencoder.py:20-369 for what the EncDiff path uses:
``VQModelInterface.encode`` (encoder + quant_conv, no quantisation, :313-316) and
``decode`` with the disentangled-representation concat (:328-369), plus the
checkpoint loader that widens post_quant_conv (:91-137).  The vector quantiser is
a state-dict-compatible restatement of taming-transformers' VectorQuantizer2
(pinned taming-transformers==0.0.1, not vendored in the reference): nearest
codebook entry, legacy beta loss, straight-through estimator.
"""
from __future__ import annotations

from contextlib import contextmanager

import torch
import torch.nn.functional as F
from torch import nn

from ..modules.diffusionmodules.model import Decoder, Encoder


class VectorQuantizer2(nn.Module):
    def __init__(self, n_e, e_dim, beta=0.25, remap=None, sane_index_shape=False, legacy=True):
        super().__init__()
        self.n_e, self.e_dim, self.beta, self.legacy = n_e, e_dim, beta, legacy
        self.sane_index_shape = sane_index_shape
        self.embedding = nn.Embedding(n_e, e_dim)
        self.embedding.weight.data.uniform_(-1.0 / n_e, 1.0 / n_e)

    def forward(self, z):
        z = z.permute(0, 2, 3, 1).contiguous()
        zf = z.view(-1, self.e_dim)
        d = (zf ** 2).sum(1, keepdim=True) + (self.embedding.weight ** 2).sum(1) - 2 * zf @ self.embedding.weight.t()
        idx = torch.argmin(d, dim=1)
        z_q = self.embedding(idx).view(z.shape)
        if self.legacy:
            loss = torch.mean((z_q.detach() - z) ** 2) + self.beta * torch.mean((z_q - z.detach()) ** 2)
        else:
            loss = self.beta * torch.mean((z_q.detach() - z) ** 2) + torch.mean((z_q - z.detach()) ** 2)
        z_q = z + (z_q - z).detach()
        z_q = z_q.permute(0, 3, 1, 2).contiguous()
        if self.sane_index_shape:
            idx = idx.reshape(z_q.shape[0], z_q.shape[2], z_q.shape[3])
        return z_q, loss, (None, None, idx)


class VQModel(nn.Module):
    def __init__(self, ddconfig, lossconfig, n_embed, embed_dim, ckpt_path=None, ignore_keys=(), image_key="image",
                 colorize_nlabels=None, monitor=None, batch_resize_range=None, scheduler_config=None,
                 lr_g_factor=1.0, remap=None, sane_index_shape=False, use_ema=False, use_disentangled_concat=False,
                 disentangled_dim=0):
        super().__init__()
        self.embed_dim, self.n_embed, self.image_key = embed_dim, n_embed, image_key
        self.use_disentangled_concat = use_disentangled_concat
        self.disentangled_dim = disentangled_dim
        self.encoder = Encoder(**ddconfig)
        self.decoder = Decoder(**ddconfig)
        self.loss = nn.Identity()  # lossconfig target is torch.nn.Identity in every EncDiff config
        self.quantize = VectorQuantizer2(n_embed, embed_dim, beta=0.25, remap=remap,
                                         sane_index_shape=sane_index_shape)
        self.quant_conv = nn.Conv2d(ddconfig["z_channels"], embed_dim, 1)
        pq_in = embed_dim + disentangled_dim if use_disentangled_concat else embed_dim
        self.post_quant_conv = nn.Conv2d(pq_in, ddconfig["z_channels"], 1)
        if monitor is not None:
            self.monitor = monitor
        if ckpt_path is not None:
            self.init_from_ckpt(ckpt_path, ignore_keys=list(ignore_keys))

    def init_from_ckpt(self, path, ignore_keys=()):
        """autoencoder.py:91-137: widen post_quant_conv when the checkpoint predates the concat."""
        sd = torch.load(path, map_location="cpu", weights_only=True)
        sd = sd.get("state_dict", sd)
        if self.use_disentangled_concat and "post_quant_conv.weight" in sd:
            old = sd["post_quant_conv.weight"]
            new_shape = self.post_quant_conv.weight.shape
            if old.shape[1] != new_shape[1]:
                w = nn.init.xavier_uniform_(torch.zeros(new_shape))
                w[:, :old.shape[1]] = old
                sd["post_quant_conv.weight"] = w
        for k in list(sd.keys()):
            if any(k.startswith(ik) for ik in ignore_keys):
                del sd[k]
        missing, unexpected = self.load_state_dict(sd, strict=False)
        print(f"Restored from {path} with {len(missing)} missing and {len(unexpected)} unexpected keys")


class VQModelInterface(VQModel):
    def __init__(self, embed_dim, *args, **kwargs):
        super().__init__(embed_dim=embed_dim, *args, **kwargs)
        self.embed_dim = embed_dim
        self._hip_encoder = None

    def enable_hip(self):
        """Route encode() through the HIP executor of the frozen encoder
        (encdiff_amd/vq.py).  Called by LatentDiffusion when it sets
        up HIP training; the module itself stays the reference's (state_dict, decode)."""
        from encdiff_amd.vq import VQEncoderExecutor
        self._hip_encoder = VQEncoderExecutor(self)
        return self

    def encode(self, x):
        if self._hip_encoder is not None:
            return self._hip_encoder.encode(x)
        return self.quant_conv(self.encoder(x))

    def decode(self, h, force_not_quantize=False, disentangled_repr=None):
        quant = h if force_not_quantize else self.quantize(h)[0]
        if self.use_disentangled_concat:
            B, _, H, W = quant.shape
            if disentangled_repr is not None:
                s = disentangled_repr[:, :, None, None].expand(-1, -1, H, W)
            else:
                s = torch.zeros(B, self.disentangled_dim, H, W, device=quant.device, dtype=quant.dtype)
            quant = torch.cat([quant, s], dim=1)
        return self.decoder(self.post_quant_conv(quant))


class IdentityFirstStage(nn.Module):
    def __init__(self, *args, vq_interface=False, **kwargs):
        super().__init__()
        self.vq_interface = vq_interface

    def encode(self, x, *args, **kwargs):
        return x

    def decode(self, x, *args, **kwargs):
        return x

    def forward(self, x, *args, **kwargs):
        return x
