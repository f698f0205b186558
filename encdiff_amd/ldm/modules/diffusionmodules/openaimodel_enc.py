"""UNetModel (the EncDiff denoiser) and the as-is concept encoder Encoder4.

Mirrors ldm/modules/diffusionmodules/openaimodel_enc.py:
  * ``UNetModel`` (:413-748): same constructor kwargs, same submodule / parameter
    names (state_dicts interchange with the reference), same forward signature
    ``forward(x, timesteps, context=[c], y=None, **kwargs)``.  The forward runs the
    MI355X executor (encdiff_amd/unet.py) through a torch.autograd.Function, so
    ``loss.backward()`` reaches the concept encoder through d(context); the UNet's
    own weight gradients are written straight into the parameter arena.
    There is no CPU path: calling it on a CPU tensor raises.
  * ``Encoder4`` / ``EncResBlock`` / ``View`` (:969-1049): plain PyTorch, called
    as-is (north_star: the concept-token image encoder is not re-implemented).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from encdiff_amd import _lib as L
from encdiff_amd import ops
from encdiff_amd.arena import ParamArena
from encdiff_amd.unet import ConvSpec, ResSpec, STSpec, UNetExecutor, UNetSpec
from ..attention import SpatialTransformer
from .util import normalization, zero_module


class TimestepBlock(nn.Module):
    pass


class TimestepEmbedSequential(nn.Sequential, TimestepBlock):
    """openaimodel_enc.py:74-88 (container; the executor walks the layers)."""


class ResBlock(TimestepBlock):
    """openaimodel_enc.py:163-275 -- parameter container with the reference names."""

    def __init__(self, channels, emb_channels, dropout, out_channels=None, use_conv=False,
                 use_scale_shift_norm=False, dims=2, use_checkpoint=False, up=False, down=False):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        self.use_scale_shift_norm = use_scale_shift_norm
        self.updown = up or down
        self.in_layers = nn.Sequential(normalization(channels), nn.SiLU(),
                                       nn.Conv2d(channels, self.out_channels, 3, padding=1))
        self.emb_layers = nn.Sequential(
            nn.SiLU(), nn.Linear(emb_channels, 2 * self.out_channels if use_scale_shift_norm else self.out_channels))
        self.out_layers = nn.Sequential(normalization(self.out_channels), nn.SiLU(), nn.Dropout(p=dropout),
                                        zero_module(nn.Conv2d(self.out_channels, self.out_channels, 3, padding=1)))
        if self.out_channels == channels:
            self.skip_connection = nn.Identity()
        elif use_conv:
            self.skip_connection = nn.Conv2d(channels, self.out_channels, 3, padding=1)
        else:
            self.skip_connection = nn.Conv2d(channels, self.out_channels, 1)

    def forward(self, x, emb):
        raise RuntimeError("ResBlock runs inside the HIP UNet executor; call UNetModel.forward")


class _UNetFn(torch.autograd.Function):
    """eps = UNet(x_t, t, context); backward returns d(context), and d(x_t) only when x_t
    requires grad (the EncDiff objective does not ask for it); weight grads go to the arena."""

    @staticmethod
    def forward(ctx, x, t, c, ex: UNetExecutor):
        ctx.ex = ex
        ctx.want_dx = bool(ctx.needs_input_grad[0])
        return ex.forward(x, t, c).clone()

    @staticmethod
    def backward(ctx, g):
        # ex.split_requested (data-parallel trainer): only the output blocks run here; the
        # d(context) buffer is filled by ex.backward_rest(), which the trainer calls itself
        ex = ctx.ex
        ex.want_dx = ctx.want_dx and not ex.split_requested
        try:
            dc = ex.backward(g.float(), split=ex.split_requested)
        finally:
            want, ex.want_dx = ex.want_dx, False
        return (ex.d_x.clone() if want else None), None, dc.clone(), None


class _UNetF32Fn(torch.autograd.Function):
    """eps = UNet(x_t, t, context) on the fp32 path (unet_f32.UNetF32): the forward saves its
    activations, the backward returns d x_t and d context and adds every UNet weight gradient
    to the arena (the parameters' .grad views)."""

    @staticmethod
    def forward(ctx, x, t, c, f32):
        ctx.f32 = f32
        return f32.forward(x, t, c, save=True)

    @staticmethod
    def backward(ctx, g):
        dx, dc = ctx.f32.backward(g.float())
        return dx, None, dc, None


_SUPPORTED = dict(dims=2, num_classes=None, use_fp16=False, num_head_channels=-1, transformer_depth=1,
                  use_spatial_transformer=True, use_scale_shift_norm=True, resblock_updown=True, n_embed=None,
                  legacy=True)


class UNetModel(nn.Module):
    """openaimodel_enc.py:413-748 for the EncDiff configuration family
    (spatial transformer, scale-shift norm, ResBlock up/down)."""

    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks,
                 attention_resolutions, latent_unit, dropout=0, channel_mult=(1, 2, 4, 8), conv_resample=True,
                 dims=2, num_classes=None, use_checkpoint=False, use_fp16=False, num_heads=-1,
                 num_head_channels=-1, num_heads_upsample=-1, use_scale_shift_norm=False, resblock_updown=False,
                 use_new_attention_order=False, use_spatial_transformer=False, transformer_depth=1,
                 context_dim=None, n_embed=None, legacy=True, attn_fp8_min_tokens=None):
        super().__init__()
        given = dict(dims=dims, num_classes=num_classes, use_fp16=use_fp16, num_head_channels=num_head_channels,
                     transformer_depth=transformer_depth, use_spatial_transformer=use_spatial_transformer,
                     use_scale_shift_norm=use_scale_shift_norm, resblock_updown=resblock_updown, n_embed=n_embed,
                     legacy=legacy)
        bad = {k: v for k, v in given.items() if v != _SUPPORTED[k]}
        if bad or dropout:
            raise NotImplementedError(f"HIP UNet path supports the EncDiff config family only; unsupported: {bad}")
        if isinstance(context_dim, (list, tuple)):
            context_dim = context_dim[0]
        self.image_size = image_size
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = list(attention_resolutions)
        self.channel_mult = list(channel_mult)
        self.num_heads = num_heads
        self.context_dim = context_dim
        self.latent_unit = latent_unit
        self.dtype = torch.float32
        self.num_classes = None
        self.predict_codebook_ids = False
        cfg = dict(image_size=image_size, in_channels=in_channels, out_channels=out_channels,
                   model_channels=model_channels, attention_resolutions=self.attention_resolutions,
                   num_res_blocks=num_res_blocks, channel_mult=self.channel_mult, num_heads=num_heads,
                   context_dim=context_dim, latent_unit=latent_unit, attn_fp8_min_tokens=attn_fp8_min_tokens)
        # attn_fp8_min_tokens (builder extension for configs[4], not a reference kwarg): self-attention
        # over >= that many tokens computes its scores on fp8 (e4m3) MFMA
        self._spec = UNetSpec.from_config(cfg)
        ted = model_channels * 4
        self.time_embed = nn.Sequential(nn.Linear(model_channels, ted), nn.SiLU(), nn.Linear(ted, ted))

        def make(layer):
            if isinstance(layer, ConvSpec):
                return nn.Conv2d(layer.cin, layer.cout, 3, padding=1)
            if isinstance(layer, ResSpec):
                return ResBlock(layer.cin, ted, 0, out_channels=layer.cout, use_scale_shift_norm=True,
                                up=layer.updown == L.RESAMPLE_UP2, down=layer.updown == L.RESAMPLE_DOWN2)
            return SpatialTransformer(layer.c, layer.heads, layer.dh, context_dim=context_dim)

        self.input_blocks = nn.ModuleList([TimestepEmbedSequential(*[make(l) for l in b])
                                           for b in self._spec.input_blocks])
        self.middle_block = TimestepEmbedSequential(*[make(l) for l in self._spec.middle])
        self.output_blocks = nn.ModuleList([TimestepEmbedSequential(*[make(l) for l in b])
                                            for b in self._spec.output_blocks])
        self.out = nn.Sequential(normalization(self._spec.out_ch), nn.SiLU(),
                                 zero_module(nn.Conv2d(model_channels, out_channels, 3, padding=1)))
        self._arena: Optional[ParamArena] = None
        self._ex: Optional[UNetExecutor] = None
        self._packed_version = -1
        self._packed_gen = -1
        # load_state_dict writes the arena through the parameters' .data views, which no
        # version counter sees: mark the bf16 packs stale explicitly
        self.register_load_state_dict_post_hook(_mark_arena_dirty)

    # ------------------------------------------------------------- HIP binding
    def bind_arena(self, arena: Optional[ParamArena] = None):
        """Put the parameters into `arena` (shared with other trainables) or a private one."""
        named = dict(self.named_parameters())
        if arena is None:
            dev = next(self.parameters()).device
            arena = ParamArena(self._spec.arena_order(named), dev, ema_names=list(named),
                               channels_last=self._spec.conv_weights())
        self._arena = arena
        self._ex = None
        return arena

    def arena_order(self):
        return self._spec.arena_order(dict(self.named_parameters()))

    def executor(self) -> UNetExecutor:
        if self._arena is None:
            self.bind_arena()
        a = self._arena
        if self._ex is None or self._ex.arena is not a:
            self._ex = UNetExecutor(self._spec, a)
            self.mark_repacked()
        elif a.master._version != self._packed_version or a.gen != self._packed_gen:
            # parameters were modified in place (arena writes, load_state_dict, EMA swap
            # -- ParamArena.mark_dirty): refresh the bf16 copies
            self._ex.pack.repack()
            self.mark_repacked()
        return self._ex

    def mark_repacked(self):
        if self._arena is not None:
            self._packed_version = self._arena.master._version
            self._packed_gen = self._arena.gen

    def forward(self, x, timesteps=None, context=None, y=None, **kwargs):
        if not x.is_cuda:
            raise RuntimeError("UNetModel runs on the MI355X HIP path only (no CPU fallback)")
        c = context[0] if isinstance(context, (list, tuple)) else context
        c = c.reshape(x.shape[0], -1).float()
        ex = self.executor()
        if getattr(self, "hip_precision", "bf16") == "fp32":
            # the reference's precision (SURVEY §8(b) convention 5): fp32 activations end to end
            # (parity checks, reference-precision sampling and gradients)
            if getattr(self, "_f32", None) is None or self._f32.ex is not ex:
                from encdiff_amd.unet_f32 import UNetF32
                self._f32 = UNetF32(ex)
            if not torch.is_grad_enabled():
                return self._f32.forward(x, timesteps, c)
            self._arena.attach_grads()
            return _UNetF32Fn.apply(x.float(), timesteps.long(), c, self._f32)
        ex.infer = not torch.is_grad_enabled()  # inference-only fusions (no saved activations)
        if ex.infer and getattr(self, "borrow_eps", False):
            # a sampler loop that consumes eps before its next call (DDIMSampler's captured loops):
            # the executor's output buffer itself, without the copy a returned tensor needs
            return ex.forward(x.float(), timesteps.long(), c)
        if torch.is_grad_enabled():
            self._arena.attach_grads()
        return _UNetFn.apply(x.float(), timesteps.long(), c, ex)


def _mark_arena_dirty(module, incompatible_keys):
    a = getattr(module, "_arena", None) or getattr(getattr(module, "_trunk", None), "arena", None)
    if a is not None:
        a.mark_dirty()


# --------------------------------------------------------------------------- Encoder4 (as-is)
class EncResBlock(nn.Module):
    """openaimodel_enc.py:969-989."""

    def __init__(self, in_channels, out_channels, mid_channels=None, bn=False):
        super().__init__()
        mid = mid_channels or out_channels
        layers = [nn.ReLU(), nn.Conv2d(in_channels, mid, 3, 1, 1), nn.ReLU(), nn.Conv2d(mid, out_channels, 1, 1, 0)]
        if bn:
            layers.insert(2, nn.BatchNorm2d(out_channels))
        self.convs = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.convs(x)


class View(nn.Module):
    def __init__(self, size):
        super().__init__()
        self.size = size

    def forward(self, tensor):
        return tensor.view(self.size)


class _WarpFn(torch.autograd.Function):
    """Encoder4.warp on encdiff_encoder_warp_fwd/bwd; weight gradients go to the arena
    directly (the module's .grad views), only d u flows back through autograd."""

    @staticmethod
    def forward(ctx, u, enc):
        arena, base, stride = enc._warp_bind
        u = u.contiguous()
        out = torch.empty(u.shape[0], enc.latent_unit * enc.context_dim, device=u.device, dtype=torch.float32)
        ops.encoder_warp_fwd(u, arena.master[base:], stride, enc.latent_unit, enc.context_dim, out)
        ctx.enc = enc
        ctx.save_for_backward(u)
        return out

    @staticmethod
    def backward(ctx, dout):
        (u,) = ctx.saved_tensors
        enc = ctx.enc
        arena, base, stride = enc._warp_bind
        du = torch.empty_like(u)
        ops.encoder_warp_bwd(u, arena.master[base:], stride, enc.latent_unit, enc.context_dim, dout.contiguous(), du,
                             arena.grad[base:])
        return du, None


def encoder4_stages(image_size: int) -> int:
    """Stride-2 stages taking an image_size^2 input down to the 4x4 grid the trunk ends on."""
    n, s = 0, image_size
    while s > 4:
        s //= 2
        n += 1
    if 4 << n != image_size or n < 2:
        raise ValueError(f"Encoder4 needs a power-of-two image_size >= 16, got {image_size}")
    return n


class Encoder4(nn.Module):
    """openaimodel_enc.py:991-1041: image -> latent_unit scalars -> per-unit MLP warp
    to context_dim-d concept tokens, concatenated to (B, latent_unit*context_dim).

    ``image_size`` (builder extension, default 64 = the reference exactly): the reference
    hard-codes four Conv2d(k4, s2, p1) stages, i.e. a 64x64 input, and View((-1, 128*4*4))
    (:1012-1013).  Other power-of-two sizes get one [Conv, BN, ReLU] stage per extra halving,
    inserted after the first (configs[4]: 128x128 CelebA -> five stages), so the trunk still ends
    on the 4x4 grid the flatten + Linear(d*16, latent_unit) expects; the second-to-last stage keeps
    the reference's BN-without-ReLU.  image_size=64 reproduces the reference module, indices and
    state_dict keys unchanged."""

    def __init__(self, d, context_dim, latent_unit, bn=True, num_channels=3, image_size=64):
        super().__init__()
        self.context_dim = context_dim
        self.latent_unit = latent_unit
        self.image_size = image_size
        n = encoder4_stages(image_size)
        layers = []
        for st in range(n):
            layers += [nn.Conv2d(num_channels if st == 0 else d, d, 4, 2, 1), nn.BatchNorm2d(d)]
            if st != n - 2:
                layers.append(nn.ReLU(True))
        layers += [EncResBlock(d, d, bn=bn), nn.BatchNorm2d(d), nn.ReLU(True), EncResBlock(d, d, bn=bn),
                   View((-1, d * 4 * 4)), nn.Linear(d * 16, latent_unit)]
        self.encoder = nn.Sequential(*layers)
        self.net = nn.ModuleList([nn.Sequential(nn.Linear(1, 64), nn.ELU(True), nn.Linear(64, 128), nn.ELU(True),
                                                nn.Linear(128, context_dim)) for _ in range(latent_unit)])
        self._warp_bind = None
        self._trunk = None
        self.register_load_state_dict_post_hook(_mark_arena_dirty)

    def bind_arena(self, arena, prefix: str):
        """Run warp() on the HIP kernels (encdiff_encoder_warp_*): the per-unit MLP
        parameters must sit in the fp32 arena contiguously, unit after unit, with one
        stride (the arena lays out named_parameters() in order, so they do); weight
        gradients are then written straight into the arena's gradient buffer."""
        sizes = [p.numel() for p in self.net[0].parameters()]
        base = arena.offsets[prefix + "net.0.0.weight"][0]
        stride = None
        for i in range(self.latent_unit):
            names = [prefix + f"net.{i}.{n}" for n, _ in self.net[i].named_parameters()]
            offs = [arena.offsets[n][0] for n in names]
            if any(o2 != o1 + s1 for o1, o2, s1 in zip(offs, offs[1:], sizes)):
                raise ValueError("Encoder4.net params are not contiguous in the arena")
            if i == 1:
                stride = offs[0] - base
            if i > 0 and offs[0] != base + i * stride:
                raise ValueError("Encoder4.net units do not have a constant arena stride")
        self._warp_bind = (arena, base, stride or sum(sizes))
        # convolution trunk on HIP when its conv weights sit channels-last in the arena
        from encdiff_amd.cond import Encoder4TrunkExecutor
        self._trunk = None
        if all(n in arena.cl for n in Encoder4TrunkExecutor.channels_last_names(self, prefix)):
            self._trunk = Encoder4TrunkExecutor(self, arena, prefix)
            self._trunk_version = (arena.master._version, arena.gen)

    def repack_hip(self):
        """Refresh the trunk's bf16 weights from the arena (after an optimizer step)."""
        if getattr(self, "_trunk", None) is not None:
            self._trunk.pack.repack()
            self._trunk_version = (self._trunk.arena.master._version, self._trunk.arena.gen)

    def _encode(self, x):
        """Trunk + Linear on HIP once the trunk is bound to the arena: training mode with
        batch-statistics BatchNorm (TrunkFn, gradients into the arena), eval mode with the
        running statistics (no gradient; the validation encoding pass).  Unbound, or on CPU
        tensors, the reference modules run."""
        ex = getattr(self, "_trunk", None)
        if ex is None or not x.is_cuda or (not self.training and torch.is_grad_enabled()):
            return self.encoder(x)
        from encdiff_amd.cond import TrunkFn
        if (ex.arena.master._version, ex.arena.gen) != self._trunk_version:  # parameters modified in place
            self.repack_hip()
        if not self.training:
            return ex.forward(x.float(), train=False, head=True).clone()
        return TrunkFn.apply(x, self.encoder[0].weight, ex)

    def warp(self, u):
        if self._warp_bind is not None:
            return _WarpFn.apply(u, self)
        return torch.cat([self.net[i](u[:, i][:, None]) for i in range(self.latent_unit)], dim=1)

    def forward(self, x):
        return self.warp(self._encode(x))

    def encoding(self, x):
        return self._encode(x)
