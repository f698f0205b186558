"""SpatialTransformer family -- parameter containers with the reference's module
names (attention.py:37-261), so state_dicts interchange with the reference.

The arithmetic of these blocks runs inside the HIP UNet executor
(encdiff_amd/unet.py: ``_st_fwd`` / ``_st_bwd``); calling a block on its own is
not a supported path and raises.
"""
from __future__ import annotations

import torch
from torch import nn


def _hip_only(name):
    raise RuntimeError(f"{name} runs inside the HIP UNet executor (encdiff_amd.unet); "
                       "call UNetModel.forward on a HIP device")


class GEGLU(nn.Module):
    """attention.py:37-44: proj C -> 2*inner; value half first, gate half second."""

    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)

    def forward(self, x):
        _hip_only("GEGLU")


class FeedForward(nn.Module):
    """attention.py:47-64 with glu=True (the only form the UNet builds)."""

    def __init__(self, dim, dim_out=None, mult=4, glu=True, dropout=0.0):
        super().__init__()
        inner = int(dim * mult)
        self.net = nn.Sequential(GEGLU(dim, inner), nn.Dropout(dropout), nn.Linear(inner, dim_out or dim))

    def forward(self, x):
        _hip_only("FeedForward")


class CrossAttention(nn.Module):
    """attention.py:152-193: q/k/v without bias, to_out Linear + Dropout.  Inside the UNet the
    executor runs it; called on its own (a HIP tensor) the attention core is
    torch.ops.encdiff.attention_fwd (MFMA flash attention, autograd through
    encdiff::attention_bwd) between bf16 projections."""

    def __init__(self, query_dim, context_dim=None, heads=8, dim_head=64, dropout=0.0):
        super().__init__()
        inner = dim_head * heads
        context_dim = query_dim if context_dim is None else context_dim
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.to_q = nn.Linear(query_dim, inner, bias=False)
        self.to_k = nn.Linear(context_dim, inner, bias=False)
        self.to_v = nn.Linear(context_dim, inner, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, query_dim), nn.Dropout(dropout))

    def forward(self, x, context=None, mask=None):
        if mask is not None:
            raise NotImplementedError("attention masks are not used by EncDiff (attention.py:185-188 unused)")
        if not x.is_cuda:
            raise RuntimeError("CrossAttention runs on the MI355X HIP path only (no CPU fallback)")
        import encdiff_amd.torch_ops  # noqa: F401  (registers torch.ops.encdiff.*)
        c = x if context is None else context
        bf = torch.bfloat16
        # q / k / v projections on the library's GEMM engine (encdiff::linear, autograd through
        # encdiff::linear_bwd), then the MFMA attention
        q = _linear(x.to(bf), self.to_q.weight.to(bf))
        k = _linear(c.to(bf), self.to_k.weight.to(bf))
        v = _linear(c.to(bf), self.to_v.weight.to(bf))
        o, _ = torch.ops.encdiff.attention_fwd(q.contiguous(), k.contiguous(), v.contiguous(), self.heads, False)
        lin, drop = self.to_out[0], self.to_out[1]
        y = _linear(o, lin.weight.to(bf)).to(x.dtype)
        return drop(y + lin.bias if lin.bias is not None else y)


def _linear(x, w):
    """x w^T on the GEMM engine (encdiff::linear).  The engine reads 16-byte rows (K, N multiples
    of 8): other widths (a context_dim or inner dim not divisible by 8) run zero-padded -- the
    padded products are exact zeros, the padding is sliced off, autograd flows through both."""
    N, K = w.shape
    kp, np_ = (-K) % 8, (-N) % 8
    if kp or np_:
        x = torch.nn.functional.pad(x, (0, kp))
        w = torch.nn.functional.pad(w, (0, kp, 0, np_))
    y = torch.ops.encdiff.linear(x.contiguous(), w.contiguous())
    return y[..., :N] if np_ else y


class BasicTransformerBlock(nn.Module):
    """attention.py:196-215."""

    def __init__(self, dim, n_heads, d_head, dropout=0.0, context_dim=None, gated_ff=True, checkpoint=True):
        super().__init__()
        self.attn1 = CrossAttention(dim, heads=n_heads, dim_head=d_head, dropout=dropout)
        self.ff = FeedForward(dim, dropout=dropout, glu=gated_ff)
        self.attn2 = CrossAttention(dim, context_dim=context_dim, heads=n_heads, dim_head=d_head, dropout=dropout)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)
        self.norm3 = nn.LayerNorm(dim)
        self.checkpoint = checkpoint  # the HIP path keeps activations (no recompute); gradients are identical

    def forward(self, x, context=None):
        _hip_only("BasicTransformerBlock")


def Normalize(in_channels):
    """attention.py:76-77."""
    return nn.GroupNorm(num_groups=32, num_channels=in_channels, eps=1e-6, affine=True)


def zero_module(module):
    for p in module.parameters():
        p.detach().zero_()
    return module


class SpatialTransformer(nn.Module):
    """attention.py:218-261 (depth 1 in every EncDiff config)."""

    def __init__(self, in_channels, n_heads, d_head, depth=1, dropout=0.0, context_dim=None):
        super().__init__()
        inner = n_heads * d_head
        self.in_channels = in_channels
        self.norm = Normalize(in_channels)
        self.proj_in = nn.Conv2d(in_channels, inner, kernel_size=1)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(inner, n_heads, d_head, dropout=dropout, context_dim=context_dim)
             for _ in range(depth)])
        self.proj_out = zero_module(nn.Conv2d(inner, in_channels, kernel_size=1))

    def forward(self, x, context=None):
        _hip_only("SpatialTransformer")
