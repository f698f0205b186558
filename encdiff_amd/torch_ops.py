"""torch.library registration of the stateless HIP ops of the path (SURVEY.md §7 / §8(b):
the reference-API modules call ``torch.ops.encdiff.*``).

Each op is a thin custom op over one C-ABI entry point (encdiff_amd.ops -> libencdiff_hip.so),
with a fake (meta) implementation so shapes propagate through FakeTensor / torch.compile
tracing without a device.  The modules use them where the reference computes the same thing
with aten ops:

  encdiff::q_sample       DDPM.q_sample                 (ddpm_enc.py:292-295)
  encdiff::l1_loss        LatentDiffusion.p_losses      (ddpm_enc.py:1194-1213): (loss, loss_vlb) + seed
  encdiff::ddim_step      DDIMSampler.p_sample_ddim     (ddim.py:188-207)
  encdiff::attention_fwd  CrossAttention core           (attention.py:170-193): (o, lse)
  encdiff::attention_bwd  its backward                  (dq, dk, dv)

The UNet itself is not an op: its forward / backward is a static schedule over an executor
that owns preallocated activation buffers and writes weight gradients into the parameter
arena (encdiff_amd/unet.py), bound to autograd by UNetModel's autograd.Function.  Every op
refuses CPU tensors (no CPU fallback).
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor
from torch.library import custom_op

from . import ops


def _dev(*ts):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("encdiff ops run on the MI355X HIP path only (no CPU fallback)")


@custom_op("encdiff::q_sample", mutates_args=())
def q_sample(x0: Tensor, noise: Tensor, t: Tensor, sqrt_ac: Tensor, sqrt_1mac: Tensor) -> Tensor:
    _dev(x0, noise, t)
    out = torch.empty_like(x0, dtype=torch.float32)
    ops.q_sample(x0.float().contiguous(), noise.float().contiguous(), t, sqrt_ac, sqrt_1mac, out)
    return out


@q_sample.register_fake
def _(x0, noise, t, sqrt_ac, sqrt_1mac):
    return torch.empty_like(x0, dtype=torch.float32)


@custom_op("encdiff::l1_loss", mutates_args=())
def l1_loss(pred: Tensor, noise: Tensor, t: Tensor, lvlb: Tensor, l_simple_weight: float) -> Tuple[Tensor, Tensor]:
    """-> (out2 = [loss, loss_vlb], seed = d loss / d pred)."""
    _dev(pred, noise, t)
    out2 = torch.empty(2, device=pred.device, dtype=torch.float32)
    seed = torch.empty_like(pred, dtype=torch.float32)
    ops.l1_loss(pred.float().contiguous(), noise.float().contiguous(), t, lvlb, out2, seed, l_simple_weight)
    return out2, seed


@l1_loss.register_fake
def _(pred, noise, t, lvlb, l_simple_weight):
    return pred.new_empty(2, dtype=torch.float32), torch.empty_like(pred, dtype=torch.float32)


@custom_op("encdiff::ddim_step", mutates_args=())
def ddim_step(x: Tensor, e: Tensor, noise: Tensor, a_t: float, a_prev: float, sigma: float,
              sqrt_one_minus_at: float) -> Tuple[Tensor, Tensor]:
    """-> (x_prev, pred_x0)."""
    _dev(x, e, noise)
    x = x.float().contiguous()
    xp, px0 = torch.empty_like(x), torch.empty_like(x)
    ops.ddim_step(x, e.float().contiguous(), noise.float().contiguous(), a_t, a_prev, sigma, sqrt_one_minus_at, xp,
                  px0)
    return xp, px0


@ddim_step.register_fake
def _(x, e, noise, a_t, a_prev, sigma, sqrt_one_minus_at):
    return torch.empty_like(x, dtype=torch.float32), torch.empty_like(x, dtype=torch.float32)


@custom_op("encdiff::attention_fwd", mutates_args=())
def attention_fwd(q: Tensor, k: Tensor, v: Tensor, heads: int, fp8: bool = False) -> Tuple[Tensor, Tensor]:
    """q (B, Sq, heads*dh), k / v (B, Sk, heads*dh) bf16 -> o (B, Sq, heads*dh) bf16,
    lse (B*heads, Sq) fp32."""
    _dev(q, k, v)
    B, sq, C = q.shape
    sk = k.shape[1]
    q2, k2, v2 = (t.reshape(-1, C).contiguous() for t in (q, k, v))
    o = torch.empty(B * sq, C, device=q.device, dtype=torch.bfloat16)
    lse = torch.empty(B * heads, sq, device=q.device, dtype=torch.float32)
    ops.attention_fwd(q2, k2, v2, o, lse, B, heads, sq, sk, C // heads, fp8=fp8)
    return o.view(B, sq, C), lse


@attention_fwd.register_fake
def _(q, k, v, heads, fp8=False):
    B, sq, C = q.shape
    return q.new_empty(B, sq, C, dtype=torch.bfloat16), q.new_empty(B * heads, sq, dtype=torch.float32)


@custom_op("encdiff::attention_bwd", mutates_args=())
def attention_bwd(q: Tensor, k: Tensor, v: Tensor, o: Tensor, lse: Tensor, d_o: Tensor, heads: int,
                  fp8: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    _dev(q, k, v, o, d_o)
    B, sq, C = q.shape
    sk = k.shape[1]
    q2, k2, v2, o2, g2 = (t.reshape(-1, C).contiguous() for t in (q, k, v, o, d_o))
    dq, dk, dv = torch.empty_like(q2), torch.empty_like(k2), torch.empty_like(v2)
    ops.attention_bwd(q2, k2, v2, o2, lse, g2, dq, dk, dv, B, heads, sq, sk, C // heads, fp8=fp8)
    return dq.view(B, sq, C), dk.view(B, sk, C), dv.view(B, sk, C)


@attention_bwd.register_fake
def _(q, k, v, o, lse, d_o, heads, fp8=False):
    return torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)


def _attn_setup(ctx, inputs, output):
    q, k, v, heads, fp8 = inputs
    o, lse = output
    ctx.save_for_backward(q, k, v, o, lse)
    ctx.heads, ctx.fp8 = heads, fp8


def _attn_backward(ctx, d_o, d_lse):
    q, k, v, o, lse = ctx.saved_tensors
    dq, dk, dv = attention_bwd(q, k, v, o, lse, d_o.to(torch.bfloat16).contiguous(), ctx.heads, ctx.fp8)
    return dq, dk, dv, None, None


attention_fwd.register_autograd(_attn_backward, setup_context=_attn_setup)


@custom_op("encdiff::linear", mutates_args=())
def linear(x: Tensor, w: Tensor) -> Tensor:
    """y = x w^T on the GEMM engine (encdiff_gemm): x (..., K) bf16, w (N, K) bf16 -> (..., N) bf16.
    The standalone CrossAttention's q / k / v projections (attention.py:159-167)."""
    _dev(x, w)
    K = x.shape[-1]
    x2 = x.reshape(-1, K).contiguous()
    y = torch.empty(x2.shape[0], w.shape[0], device=x.device, dtype=torch.bfloat16)
    ops.linear_fwd(x2, w.contiguous(), y)
    return y.view(*x.shape[:-1], w.shape[0])


@linear.register_fake
def _(x, w):
    return x.new_empty(*x.shape[:-1], w.shape[0], dtype=torch.bfloat16)


@custom_op("encdiff::linear_bwd", mutates_args=())
def linear_bwd(dy: Tensor, x: Tensor, w: Tensor) -> Tuple[Tensor, Tensor]:
    """-> (dx = dy w (bf16), dw = dy^T x (fp32)): the input and weight gradient GEMMs."""
    _dev(dy, x, w)
    N, K = w.shape
    dy2, x2 = dy.reshape(-1, N).contiguous(), x.reshape(-1, K).contiguous()
    dx = torch.empty_like(x2)
    dw = torch.zeros(N, K, device=w.device, dtype=torch.float32)
    ops.linear_bwd(dy2, w.contiguous(), x2, dx, dw)
    ops.flush()
    return dx.view(x.shape), dw


@linear_bwd.register_fake
def _(dy, x, w):
    return torch.empty_like(x), w.new_empty(w.shape, dtype=torch.float32)


def _linear_setup(ctx, inputs, output):
    x, w = inputs
    ctx.save_for_backward(x, w)


def _linear_backward(ctx, dy):
    x, w = ctx.saved_tensors
    dx, dw = linear_bwd(dy.to(torch.bfloat16).contiguous(), x, w)
    return dx, dw.to(w.dtype)


linear.register_autograd(_linear_backward, setup_context=_linear_setup)
