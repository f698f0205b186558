"""CPU oracle for the EncDiff denoising path -- TEST INFRASTRUCTURE ONLY.

This module is a functional, CPU-only restatement of the reference algorithm
(SelenaGeRuiqi/EncDiff, mounted read-only at /root/reference when the fixtures
were generated).  It is the *checker*: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  The product path
(``encdiff_amd``) never imports, links or executes anything under ``oracle/``.

Parity pinning: ``tests/golden/*.npz`` were produced by ``tools/gen_golden.py``
which imports the reference's own modules (with import shims for absent
third-party packages) and runs them on the same deterministic weights and
inputs; ``tests/test_oracle_golden.py`` checks this restatement against those
fixtures.  Numerics: plain torch fp32 (or fp64 on request), same op order as
the reference.

Every function cites the reference file:line it restates.
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------
# Architecture plan (restates the constructor logic of
# ldm/modules/diffusionmodules/openaimodel_enc.py:443-688)
# ----------------------------------------------------------------------------

SHAPES3D_UNET = dict(image_size=16, in_channels=3, out_channels=3, model_channels=64,
                     attention_resolutions=[1, 2, 4], num_res_blocks=2,
                     channel_mult=[1, 2, 4, 4], num_heads=8, use_scale_shift_norm=True,
                     resblock_updown=True, use_spatial_transformer=True, context_dim=16,
                     latent_unit=20)


@dataclass
class Layer:
    kind: str            # 'conv' | 'res' | 'st'
    cin: int = 0
    cout: int = 0
    updown: str = ''     # '' | 'down' | 'up'
    heads: int = 0
    dh: int = 0
    fp8_min_tokens: int = 0  # st: self-attention scores in e4m3 from this many tokens (configs[4])


@dataclass
class Plan:
    cfg: dict
    input_blocks: List[List[Layer]] = field(default_factory=list)
    middle: List[Layer] = field(default_factory=list)
    output_blocks: List[List[Layer]] = field(default_factory=list)
    out_ch: int = 0


def build_plan(cfg: dict = SHAPES3D_UNET) -> Plan:
    """openaimodel_enc.py:507-688 (legacy=True, use_spatial_transformer=True,
    num_head_channels=-1, transformer_depth=1)."""
    mc = cfg['model_channels']
    heads = cfg['num_heads']
    attn = cfg['attention_resolutions']
    nrb = cfg['num_res_blocks']
    mult = cfg['channel_mult']
    f8 = cfg.get('attn_fp8_min_tokens') or 0
    p = Plan(cfg=cfg)
    p.input_blocks.append([Layer('conv', cfg['in_channels'], mc)])
    chans = [mc]
    ch, ds = mc, 1
    for level, m in enumerate(mult):
        for _ in range(nrb):
            blk = [Layer('res', ch, m * mc)]
            ch = m * mc
            if ds in attn:
                blk.append(Layer('st', ch, ch, heads=heads, dh=ch // heads, fp8_min_tokens=f8))
            p.input_blocks.append(blk)
            chans.append(ch)
        if level != len(mult) - 1:
            p.input_blocks.append([Layer('res', ch, ch, updown='down')])
            chans.append(ch)
            ds *= 2
    p.middle = [Layer('res', ch, ch), Layer('st', ch, ch, heads=heads, dh=ch // heads, fp8_min_tokens=f8),
                Layer('res', ch, ch)]
    for level, m in list(enumerate(mult))[::-1]:
        for i in range(nrb + 1):
            ich = chans.pop()
            blk = [Layer('res', ch + ich, mc * m)]
            ch = mc * m
            if ds in attn:
                blk.append(Layer('st', ch, ch, heads=heads, dh=ch // heads, fp8_min_tokens=f8))
            if level and i == nrb:
                blk.append(Layer('res', ch, ch, updown='up'))
                ds //= 2
            p.output_blocks.append(blk)
    p.out_ch = ch
    return p


def param_shapes(plan: Plan) -> Dict[str, Tuple[int, ...]]:
    """Reference state_dict names/shapes of UNetModel (openaimodel_enc.py:507-688,
    attention.py:152-261)."""
    cfg = plan.cfg
    mc = cfg['model_channels']
    ted = 4 * mc
    cd = cfg['context_dim']
    S: Dict[str, Tuple[int, ...]] = {}
    S['time_embed.0.weight'] = (ted, mc); S['time_embed.0.bias'] = (ted,)
    S['time_embed.2.weight'] = (ted, ted); S['time_embed.2.bias'] = (ted,)

    def layer_shapes(pre: str, L: Layer):
        if L.kind == 'conv':
            S[pre + 'weight'] = (L.cout, L.cin, 3, 3); S[pre + 'bias'] = (L.cout,)
        elif L.kind == 'res':
            S[pre + 'in_layers.0.weight'] = (L.cin,); S[pre + 'in_layers.0.bias'] = (L.cin,)
            S[pre + 'in_layers.2.weight'] = (L.cout, L.cin, 3, 3); S[pre + 'in_layers.2.bias'] = (L.cout,)
            S[pre + 'emb_layers.1.weight'] = (2 * L.cout, ted); S[pre + 'emb_layers.1.bias'] = (2 * L.cout,)
            S[pre + 'out_layers.0.weight'] = (L.cout,); S[pre + 'out_layers.0.bias'] = (L.cout,)
            S[pre + 'out_layers.3.weight'] = (L.cout, L.cout, 3, 3); S[pre + 'out_layers.3.bias'] = (L.cout,)
            if L.cin != L.cout:
                S[pre + 'skip_connection.weight'] = (L.cout, L.cin, 1, 1)
                S[pre + 'skip_connection.bias'] = (L.cout,)
        else:
            c = L.cin
            S[pre + 'norm.weight'] = (c,); S[pre + 'norm.bias'] = (c,)
            S[pre + 'proj_in.weight'] = (c, c, 1, 1); S[pre + 'proj_in.bias'] = (c,)
            t = pre + 'transformer_blocks.0.'
            for a, kv in (('attn1', c), ('attn2', cd)):
                S[t + a + '.to_q.weight'] = (c, c)
                S[t + a + '.to_k.weight'] = (c, kv)
                S[t + a + '.to_v.weight'] = (c, kv)
                S[t + a + '.to_out.0.weight'] = (c, c); S[t + a + '.to_out.0.bias'] = (c,)
            S[t + 'ff.net.0.proj.weight'] = (8 * c, c); S[t + 'ff.net.0.proj.bias'] = (8 * c,)
            S[t + 'ff.net.2.weight'] = (c, 4 * c); S[t + 'ff.net.2.bias'] = (c,)
            for n in ('norm1', 'norm2', 'norm3'):
                S[t + n + '.weight'] = (c,); S[t + n + '.bias'] = (c,)
            S[pre + 'proj_out.weight'] = (c, c, 1, 1); S[pre + 'proj_out.bias'] = (c,)

    for i, blk in enumerate(plan.input_blocks):
        for j, L in enumerate(blk):
            layer_shapes(f'input_blocks.{i}.{j}.', L)
    for j, L in enumerate(plan.middle):
        layer_shapes(f'middle_block.{j}.', L)
    for i, blk in enumerate(plan.output_blocks):
        for j, L in enumerate(blk):
            layer_shapes(f'output_blocks.{i}.{j}.', L)
    S['out.0.weight'] = (plan.out_ch,); S['out.0.bias'] = (plan.out_ch,)
    S['out.2.weight'] = (cfg['out_channels'], mc, 3, 3); S['out.2.bias'] = (cfg['out_channels'],)
    return S


# ----------------------------------------------------------------------------
# Deterministic weight recipe shared by fixtures and tests (no weights are
# committed: they are regenerated from the tensor name).
# ----------------------------------------------------------------------------

def recipe_tensor(name: str, shape: Tuple[int, ...], seed: int = 0) -> torch.Tensor:
    """Counter-based init: generator seeded by crc32(name) ^ seed.  Every tensor
    is non-zero (zero-init layers of the reference would make eps == 0)."""
    g = torch.Generator().manual_seed((zlib.crc32(name.encode()) ^ seed) & 0x7FFFFFFF)
    z = torch.randn(shape, generator=g, dtype=torch.float64)
    leaf = name.rsplit('.', 1)[-1]
    if len(shape) == 1:
        is_norm = any(k in name for k in ('norm', 'in_layers.0', 'out_layers.0', 'out.0'))
        if leaf == 'weight' and is_norm:
            return (1.0 + 0.1 * z).float()
        return (0.05 * z).float()
    fan_in = int(np.prod(shape[1:]))
    return (z / math.sqrt(fan_in)).float()


def recipe_params(shapes: Dict[str, Tuple[int, ...]], seed: int = 0) -> Dict[str, torch.Tensor]:
    return {k: recipe_tensor(k, v, seed) for k, v in shapes.items()}


# ----------------------------------------------------------------------------
# Functional UNet (openaimodel_enc.py:163-275, 712-748; attention.py:37-261;
# util.py:179-199, 242-244)
# ----------------------------------------------------------------------------

def timestep_embedding(t: torch.Tensor, dim: int, max_period: int = 10000) -> torch.Tensor:
    """util.py:179-199: cat[cos(t f), sin(t f)], f_k = exp(-ln(max_period) k / half)."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    return torch.cat([torch.cos(args), torch.sin(args)], dim=-1)


def group_norm32(x, w, b, eps=1e-5):
    """util.py:242-244 GroupNorm32: 32 groups, fp32 compute."""
    return F.group_norm(x.float(), 32, w, b, eps).type(x.dtype)


def resblock(P, pre, L: Layer, x, emb):
    """openaimodel_enc.py:255-275 (use_scale_shift_norm=True)."""
    h = F.silu(group_norm32(x, P[pre + 'in_layers.0.weight'], P[pre + 'in_layers.0.bias']))
    if L.updown == 'down':                       # :256-261, Downsample(use_conv=False) :156
        h = F.avg_pool2d(h, 2, 2)
        x = F.avg_pool2d(x, 2, 2)
    elif L.updown == 'up':                       # Upsample :116
        h = F.interpolate(h, scale_factor=2, mode='nearest')
        x = F.interpolate(x, scale_factor=2, mode='nearest')
    h = F.conv2d(h, P[pre + 'in_layers.2.weight'], P[pre + 'in_layers.2.bias'], padding=1)
    e = F.linear(F.silu(emb), P[pre + 'emb_layers.1.weight'], P[pre + 'emb_layers.1.bias'])
    scale, shift = torch.chunk(e[:, :, None, None], 2, dim=1)
    h = group_norm32(h, P[pre + 'out_layers.0.weight'], P[pre + 'out_layers.0.bias']) * (1 + scale) + shift
    h = F.conv2d(F.silu(h), P[pre + 'out_layers.3.weight'], P[pre + 'out_layers.3.bias'], padding=1)
    if L.cin != L.cout:
        x = F.conv2d(x, P[pre + 'skip_connection.weight'], P[pre + 'skip_connection.bias'])
    return x + h


class _FP8Scores(torch.autograd.Function):
    """q k^T with q, k rounded to OCP e4m3 (torch.float8_e4m3fn) -- the builder's configs[4]
    fp8 self-attention scores (no reference counterpart: the reference is fp32).  The backward
    uses the unrounded q, k, as the HIP kernel's dQ = dS K and dK = dS^T Q products do."""

    @staticmethod
    def forward(ctx, q, k):
        ctx.save_for_backward(q, k)
        e4 = torch.float8_e4m3fn
        return torch.einsum('bid,bjd->bij', q.to(e4).float(), k.to(e4).float())

    @staticmethod
    def backward(ctx, g):
        q, k = ctx.saved_tensors
        return torch.einsum('bij,bjd->bid', g, k), torch.einsum('bij,bid->bjd', g, q)


def cross_attention(P, pre, x, ctx, heads, fp8=False):
    """attention.py:170-193: q,k,v no bias; softmax(q k^T * dh^-0.5) v; to_out.
    fp8: scores from e4m3-rounded q, k (configs[4]'s long-sequence self-attention)."""
    q = F.linear(x, P[pre + 'to_q.weight'])
    c = x if ctx is None else ctx
    k = F.linear(c, P[pre + 'to_k.weight'])
    v = F.linear(c, P[pre + 'to_v.weight'])
    b, n, inner = q.shape
    dh = inner // heads

    def split(t):  # 'b n (h d) -> (b h) n d'
        return t.reshape(t.shape[0], t.shape[1], heads, dh).permute(0, 2, 1, 3).reshape(-1, t.shape[1], dh)
    q, k, v = split(q), split(k), split(v)
    sim = (_FP8Scores.apply(q, k) if fp8 else torch.einsum('bid,bjd->bij', q, k)) * (dh ** -0.5)
    attn = sim.softmax(dim=-1)
    out = torch.einsum('bij,bjd->bid', attn, v)
    out = out.reshape(b, heads, n, dh).permute(0, 2, 1, 3).reshape(b, n, inner)
    return F.linear(out, P[pre + 'to_out.0.weight'], P[pre + 'to_out.0.bias'])


def spatial_transformer(P, pre, L: Layer, x, ctx):
    """attention.py:250-261 + BasicTransformerBlock._forward :211-215 + GEGLU :37-64."""
    b, c, hh, ww = x.shape
    x_in = x
    x = F.group_norm(x, 32, P[pre + 'norm.weight'], P[pre + 'norm.bias'], 1e-6)
    x = F.conv2d(x, P[pre + 'proj_in.weight'], P[pre + 'proj_in.bias'])
    x = x.permute(0, 2, 3, 1).reshape(b, hh * ww, c)
    t = pre + 'transformer_blocks.0.'
    ln = lambda y, n: F.layer_norm(y, (c,), P[t + n + '.weight'], P[t + n + '.bias'], 1e-5)
    fp8_min = L.fp8_min_tokens
    x = cross_attention(P, t + 'attn1.', ln(x, 'norm1'), None, L.heads, fp8=bool(fp8_min) and hh * ww >= fp8_min) + x
    x = cross_attention(P, t + 'attn2.', ln(x, 'norm2'), ctx, L.heads) + x
    y = F.linear(ln(x, 'norm3'), P[t + 'ff.net.0.proj.weight'], P[t + 'ff.net.0.proj.bias'])
    a, g = y.chunk(2, dim=-1)
    y = F.linear(a * F.gelu(g), P[t + 'ff.net.2.weight'], P[t + 'ff.net.2.bias'])
    x = y + x
    x = x.reshape(b, hh, ww, c).permute(0, 3, 1, 2)
    x = F.conv2d(x, P[pre + 'proj_out.weight'], P[pre + 'proj_out.bias'])
    return x + x_in


def unet_forward(P: Dict[str, torch.Tensor], plan: Plan, x, timesteps, context):
    """openaimodel_enc.py:712-748.  ``context`` is the list-wrapped (B, latent_unit*context_dim)
    tensor or the bare tensor."""
    cfg = plan.cfg
    if isinstance(context, (list, tuple)):
        context = context[0]
    b = x.shape[0]
    emb = timestep_embedding(timesteps, cfg['model_channels'])
    emb = F.linear(emb, P['time_embed.0.weight'], P['time_embed.0.bias'])
    emb = F.linear(F.silu(emb), P['time_embed.2.weight'], P['time_embed.2.bias'])
    ctx = context.reshape(b, -1, cfg['context_dim'])

    def run(pre, L, h):
        if L.kind == 'conv':
            return F.conv2d(h, P[pre + 'weight'], P[pre + 'bias'], padding=1)
        if L.kind == 'res':
            return resblock(P, pre, L, h, emb)
        return spatial_transformer(P, pre, L, h, ctx)

    hs = []
    h = x
    for i, blk in enumerate(plan.input_blocks):
        for j, L in enumerate(blk):
            h = run(f'input_blocks.{i}.{j}.', L, h)
        hs.append(h)
    for j, L in enumerate(plan.middle):
        h = run(f'middle_block.{j}.', L, h)
    for i, blk in enumerate(plan.output_blocks):
        h = torch.cat([h, hs.pop()], dim=1)
        for j, L in enumerate(blk):
            h = run(f'output_blocks.{i}.{j}.', L, h)
    h = F.silu(group_norm32(h, P['out.0.weight'], P['out.0.bias']))
    return F.conv2d(h, P['out.2.weight'], P['out.2.bias'], padding=1)


# ----------------------------------------------------------------------------
# Diffusion schedule, q_sample, p_losses (ddpm_enc.py:133-187, 292-310, 1183-1253;
# util.py:21-25)
# ----------------------------------------------------------------------------

def register_schedule(timesteps=1000, linear_start=0.0015, linear_end=0.0155):
    """ddpm_enc.py:133-187 with make_beta_schedule('linear') util.py:21-25.
    Returns fp64 numpy arrays (the reference casts them to fp32 buffers)."""
    betas = np.linspace(linear_start ** 0.5, linear_end ** 0.5, timesteps, dtype=np.float64) ** 2
    alphas = 1.0 - betas
    ac = np.cumprod(alphas, axis=0)
    ac_prev = np.append(1.0, ac[:-1])
    ac_next = np.append(ac[1:], ac[-1])
    post_var = betas * (1.0 - ac_prev) / (1.0 - ac)
    d = dict(betas=betas, alphas_cumprod=ac, alphas_cumprod_prev=ac_prev,
             alphas_cumprod_next=ac_next, sqrt_alphas_cumprod=np.sqrt(ac),
             sqrt_one_minus_alphas_cumprod=np.sqrt(1.0 - ac),
             log_one_minus_alphas_cumprod=np.log(1.0 - ac),
             sqrt_recip_alphas_cumprod=np.sqrt(1.0 / ac),
             sqrt_recipm1_alphas_cumprod=np.sqrt(1.0 / ac - 1),
             posterior_variance=post_var,
             posterior_log_variance_clipped=np.log(np.maximum(post_var, 1e-20)),
             posterior_mean_coef1=betas * np.sqrt(ac_prev) / (1.0 - ac),
             posterior_mean_coef2=(1.0 - ac_prev) * np.sqrt(alphas) / (1.0 - ac))
    # lvlb_weights (eps parameterisation) computed on fp32 buffers as the reference does (:176-185)
    b32 = torch.tensor(betas, dtype=torch.float32)
    pv32 = torch.tensor(post_var, dtype=torch.float32)
    a32 = torch.tensor(alphas, dtype=torch.float32)
    ac32 = torch.tensor(ac, dtype=torch.float32)
    lv = b32 ** 2 / (2 * pv32 * a32 * (1 - ac32))
    lv[0] = lv[1]
    d['lvlb_weights'] = lv.numpy().astype(np.float64)
    return d


def q_sample(sched32: Dict[str, torch.Tensor], x0, t, noise):
    """ddpm_enc.py:292-295 (+ extract_into_tensor util.py:124-127)."""
    a = sched32['sqrt_alphas_cumprod'].gather(-1, t).reshape(-1, 1, 1, 1)
    s = sched32['sqrt_one_minus_alphas_cumprod'].gather(-1, t).reshape(-1, 1, 1, 1)
    return a * x0 + s * noise


def p_losses_from_output(sched32, model_out, noise, t, logvar=None, l_simple_weight=1.0,
                         original_elbo_weight=0.0):
    """ddpm_enc.py:1194-1216 (eps parameterisation, loss_type l1, logvar == 0)."""
    loss_simple = (noise - model_out).abs().mean([1, 2, 3])
    if logvar is None:
        logvar = torch.zeros(1000)
    logvar_t = logvar[t]
    loss = loss_simple / torch.exp(logvar_t) + logvar_t
    loss = l_simple_weight * loss.mean()
    loss_vlb = (sched32['lvlb_weights'][t] * (noise - model_out).abs().mean(dim=(1, 2, 3))).mean()
    loss = loss + original_elbo_weight * loss_vlb
    return loss, {'loss_simple': loss_simple.mean(), 'loss_vlb': loss_vlb, 'loss': loss}


def sched_fp32(d):
    return {k: torch.tensor(v, dtype=torch.float32) for k, v in d.items()}


# ----------------------------------------------------------------------------
# DDIM (ddim.py:24-54, 114-207; util.py:73-102)
# ----------------------------------------------------------------------------

def ddim_schedule(alphas_cumprod32: torch.Tensor, S: int, eta: float, num_ddpm=1000):
    """make_ddim_timesteps('uniform') util.py:73-87 + make_ddim_sampling_parameters util.py:90-102.
    alphacums is the fp32 buffer moved to numpy, as in ddim.py:43-45."""
    c = num_ddpm // S
    ts = np.asarray(list(range(0, num_ddpm, c))) + 1
    # same mixed torch-fp32 / numpy-fp64 expression as the reference (util.py:92-96)
    ac = alphas_cumprod32.cpu()
    alphas = ac[ts]
    alphas_prev = np.asarray([ac[0]] + ac[ts[:-1]].tolist())
    sigmas = eta * np.sqrt((1 - alphas_prev) / (1 - alphas) * (1 - alphas / alphas_prev))
    f64 = lambda a: np.asarray(a.numpy() if isinstance(a, torch.Tensor) else a, dtype=np.float64)
    alphas = f64(alphas)
    return dict(timesteps=ts, alphas=alphas, alphas_prev=f64(alphas_prev), sigmas=f64(sigmas),
                sqrt_one_minus_alphas=np.sqrt(1.0 - alphas))


def ddim_step(x, e_t, a_t, a_prev, sigma_t, sqrt_one_minus_at, noise):
    """ddim.py:188-207 (no quantize, temperature 1, no noise dropout); the
    reference builds the four scalars with torch.full(..., float32)."""
    a_t = torch.tensor(a_t, dtype=torch.float32)
    a_prev = torch.tensor(a_prev, dtype=torch.float32)
    sigma_t = torch.tensor(sigma_t, dtype=torch.float32)
    s1 = torch.tensor(sqrt_one_minus_at, dtype=torch.float32)
    pred_x0 = (x - s1 * e_t) / a_t.sqrt()
    dir_xt = (1.0 - a_prev - sigma_t ** 2).sqrt() * e_t
    x_prev = a_prev.sqrt() * pred_x0 + dir_xt + sigma_t * noise
    return x_prev, pred_x0


def ddim_sample(eps_fn, x_T, S, eta, alphas_cumprod32, noise_fn=torch.randn, log_every_t=None):
    """ddim.py:114-166: iterate flip(timesteps); index = S - i - 1.  With ``log_every_t`` also
    returns the reference's intermediates dict (x_inter / pred_x0 logged at index %
    log_every_t == 0 or index == S - 1, after x_T itself; ddim.py:132-166)."""
    d = ddim_schedule(alphas_cumprod32, S, eta)
    x = x_T
    b = x.shape[0]
    inter = {'x_inter': [x_T], 'pred_x0': [x_T]}
    for i, step in enumerate(np.flip(d['timesteps'])):
        index = S - i - 1
        ts = torch.full((b,), int(step), dtype=torch.long)
        e_t = eps_fn(x, ts)
        noise = noise_fn(x.shape)
        x, px0 = ddim_step(x, e_t, d['alphas'][index], d['alphas_prev'][index], d['sigmas'][index],
                           d['sqrt_one_minus_alphas'][index], noise)
        if log_every_t and (index % log_every_t == 0 or index == S - 1):
            inter['x_inter'].append(x)
            inter['pred_x0'].append(px0)
    return (x, inter) if log_every_t else x


# ----------------------------------------------------------------------------
# EMA (ema.py:25-44), AdamW (torch defaults, ddpm_enc.py:1615), LR schedule
# (lr_scheduler.py:81-97)
# ----------------------------------------------------------------------------

def ema_update(shadow: Dict[str, torch.Tensor], params: Dict[str, torch.Tensor], num_updates: int,
               decay: float = 0.9999):
    """ema.py:25-44.  Returns (new_shadow, new_num_updates)."""
    num_updates += 1
    d = min(decay, (1 + num_updates) / (10 + num_updates))
    omd = 1.0 - torch.tensor(d, dtype=torch.float32)  # decay buffer is fp32; python min keeps fp32 tensor
    out = {k: s - omd * (s - params[k]) for k, s in shadow.items()}
    return out, num_updates


def adamw_step(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, wd=1e-2):
    """torch.optim.AdamW single-tensor update (torch defaults)."""
    p = p * (1 - lr * wd)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def lambda_linear_schedule(n, warm_up_steps=(10000,), f_start=(1e-6,), f_max=(1.0,), f_min=(1.0,),
                           cycle_lengths=(10000000000000,)):
    """lr_scheduler.py:81-97 (LambdaLinearScheduler.schedule)."""
    cum = np.cumsum([0] + list(cycle_lengths))
    cycle = 0
    for i, cl in enumerate(cum[1:]):
        if n <= cl:
            cycle = i
            break
    n = n - cum[cycle]
    if n < warm_up_steps[cycle]:
        return (f_max[cycle] - f_start[cycle]) / warm_up_steps[cycle] * n + f_start[cycle]
    return f_min[cycle] + (f_max[cycle] - f_min[cycle]) * (cycle_lengths[cycle] - n) / cycle_lengths[cycle]


# ----------------------------------------------------------------------------
# Concept-token encoder Encoder4 (openaimodel_enc.py:969-1049), functional.
# ----------------------------------------------------------------------------

def encoder4_layout(image_size=64):
    """Indices of Encoder4.encoder (openaimodel_enc.py:996-1013): the stride-2 stages as
    (conv, bn, relu), the two EncResBlocks with their following BN (or None), the Linear.
    The reference is image_size 64 (four stages); the builder's 128x128 variant (configs[4])
    inserts one more [Conv, BN, ReLU] stage after the first (Encoder4 image_size in the build)."""
    n, sz = 0, image_size
    while sz > 4:
        sz //= 2
        n += 1
    stages, i = [], 0
    for st in range(n):
        relu = st != n - 2
        stages.append((i, i + 1, relu))
        i += 3 if relu else 2
    res = [(i, i + 1), (i + 3, None)]
    return stages, res, i + 5


def encoder4_shapes(d=128, context_dim=16, latent_unit=20, num_channels=3, image_size=64):
    S = {}
    e = 'encoder.'
    stages, res, lin = encoder4_layout(image_size)

    def bn(i):
        for n, sh in (('weight', (d,)), ('bias', (d,)), ('running_mean', (d,)), ('running_var', (d,)),
                      ('num_batches_tracked', ())):
            S[e + f'{i}.{n}'] = sh
    for k, (ci, bi, _) in enumerate(stages):
        S[e + f'{ci}.weight'] = (d, num_channels if k == 0 else d, 4, 4); S[e + f'{ci}.bias'] = (d,)
        bn(bi)
    for ri, bi in res:
        S[e + f'{ri}.convs.1.weight'] = (d, d, 3, 3); S[e + f'{ri}.convs.1.bias'] = (d,)
        for n, sh in (('weight', (d,)), ('bias', (d,)), ('running_mean', (d,)), ('running_var', (d,)),
                      ('num_batches_tracked', ())):
            S[e + f'{ri}.convs.2.{n}'] = sh
        S[e + f'{ri}.convs.4.weight'] = (d, d, 1, 1); S[e + f'{ri}.convs.4.bias'] = (d,)
        if bi is not None:
            bn(bi)
    S[e + f'{lin}.weight'] = (latent_unit, d * 16); S[e + f'{lin}.bias'] = (latent_unit,)
    for u in range(latent_unit):
        S[f'net.{u}.0.weight'] = (64, 1); S[f'net.{u}.0.bias'] = (64,)
        S[f'net.{u}.2.weight'] = (128, 64); S[f'net.{u}.2.bias'] = (128,)
        S[f'net.{u}.4.weight'] = (context_dim, 128); S[f'net.{u}.4.bias'] = (context_dim,)
    return S


def encoder4_params(seed=0, **kw):
    S = encoder4_shapes(**kw)
    P = {}
    for k, sh in S.items():
        if k.endswith('num_batches_tracked'):
            P[k] = torch.tensor(0, dtype=torch.long)
        elif k.endswith('running_mean'):
            P[k] = torch.zeros(sh)
        elif k.endswith('running_var'):
            P[k] = torch.ones(sh)
        else:
            P[k] = recipe_tensor('cond.' + k, sh, seed)
    return P


def encoder4_forward(P, x, latent_unit=20, train=True, return_u=False):
    """openaimodel_enc.py:996-1031 (BatchNorm in train mode uses batch stats, eval mode the
    running statistics).  return_u: also the scalar codes u = encoding(x) (:1034-1035).
    The stage count follows the input resolution (reference: 64x64, four stages)."""
    e = 'encoder.'
    stages, res, lin = encoder4_layout(x.shape[-1])

    def bn(h, i):
        return F.batch_norm(h, P[e + f'{i}.running_mean'].clone(), P[e + f'{i}.running_var'].clone(),
                            P[e + f'{i}.weight'], P[e + f'{i}.bias'], training=train, momentum=0.1, eps=1e-5)

    def conv(h, i, s=2, p=1):
        return F.conv2d(h, P[e + f'{i}.weight'], P[e + f'{i}.bias'], stride=s, padding=p)

    def encres(h, i):
        y = F.relu(h)
        y = F.conv2d(y, P[e + f'{i}.convs.1.weight'], P[e + f'{i}.convs.1.bias'], padding=1)
        y = F.batch_norm(y, P[e + f'{i}.convs.2.running_mean'].clone(), P[e + f'{i}.convs.2.running_var'].clone(),
                         P[e + f'{i}.convs.2.weight'], P[e + f'{i}.convs.2.bias'], training=train, momentum=0.1,
                         eps=1e-5)
        y = F.relu(y)
        y = F.conv2d(y, P[e + f'{i}.convs.4.weight'], P[e + f'{i}.convs.4.bias'])
        return h + y

    h = x
    for ci, bi, relu in stages:
        h = bn(conv(h, ci), bi)
        if relu:
            h = F.relu(h)
    (r0, b0), (r1, _) = res
    h = F.relu(bn(encres(h, r0), b0))
    h = encres(h, r1)
    d = h.shape[1]
    h = h.reshape(-1, d * 4 * 4)
    u = F.linear(h, P[e + f'{lin}.weight'], P[e + f'{lin}.bias'])
    c = encoder4_warp(P, u, latent_unit)
    return (c, u) if return_u else c


def encoder4_warp(P, u, latent_unit=20):
    """Encoder4.warp (openaimodel_enc.py:1037-1041): unit i's scalar code through its own
    Linear(1, 64) ELU Linear(64, 128) ELU Linear(128, context_dim); tokens concatenated."""
    outs = []
    for i in range(latent_unit):
        y = u[:, i][:, None]
        y = F.elu(F.linear(y, P[f'net.{i}.0.weight'], P[f'net.{i}.0.bias']))
        y = F.elu(F.linear(y, P[f'net.{i}.2.weight'], P[f'net.{i}.2.bias']))
        outs.append(F.linear(y, P[f'net.{i}.4.weight'], P[f'net.{i}.4.bias']))
    return torch.cat(outs, dim=1)


# ----------------------------------------------------------------------------
# Frozen VQ first-stage encoder (VQModelInterface.encode, autoencoder.py:313-316 =
# quant_conv(Encoder(x)); Encoder model.py:368-459, ResnetBlock :82-141, AttnBlock
# :150-200, Downsample :60-80, Normalize :38-39 (GroupNorm 32, eps 1e-6),
# nonlinearity :33-35 (x * sigmoid(x))), functional.  Parameter names are the
# first_stage_model state_dict names.
# ----------------------------------------------------------------------------

VQ_F4 = dict(ch=32, ch_mult=(1, 2, 4), num_res_blocks=2, attn_resolutions=(), in_channels=3, z_channels=3,
             embed_dim=3, resolution=64)  # shapes3d-vq-4-16-encdiff.yaml first_stage_config


def vq_encoder_shapes(cfg=VQ_F4) -> Dict[str, Tuple[int, ...]]:
    S: Dict[str, Tuple[int, ...]] = {}

    def conv(pre, co, ci, k):
        S[pre + 'weight'] = (co, ci, k, k)
        S[pre + 'bias'] = (co,)

    def norm(pre, c):
        S[pre + 'weight'] = (c,)
        S[pre + 'bias'] = (c,)

    def resnet(pre, ci, co):  # model.py:82-119 (temb_channels = 0: no temb_proj)
        norm(pre + 'norm1.', ci)
        conv(pre + 'conv1.', co, ci, 3)
        norm(pre + 'norm2.', co)
        conv(pre + 'conv2.', co, co, 3)
        if ci != co:
            conv(pre + 'nin_shortcut.', co, ci, 1)

    def attn(pre, c):  # model.py:150-176
        norm(pre + 'norm.', c)
        for n in ('q', 'k', 'v', 'proj_out'):
            conv(pre + n + '.', c, c, 1)

    ch, mult = cfg['ch'], tuple(cfg['ch_mult'])
    conv('encoder.conv_in.', ch, cfg['in_channels'], 3)
    in_mult = (1,) + mult
    curr = cfg['resolution']
    bi = ch
    for i, m in enumerate(mult):  # model.py:386-408
        bi, bo = ch * in_mult[i], ch * m
        for j in range(cfg['num_res_blocks']):
            resnet(f'encoder.down.{i}.block.{j}.', bi, bo)
            bi = bo
            if curr in cfg['attn_resolutions']:
                attn(f'encoder.down.{i}.attn.{j}.', bi)
        if i != len(mult) - 1:
            conv(f'encoder.down.{i}.downsample.conv.', bi, bi, 3)
            curr //= 2
    resnet('encoder.mid.block_1.', bi, bi)
    attn('encoder.mid.attn_1.', bi)
    resnet('encoder.mid.block_2.', bi, bi)
    norm('encoder.norm_out.', bi)
    conv('encoder.conv_out.', cfg['z_channels'], bi, 3)
    conv('quant_conv.', cfg['embed_dim'], cfg['z_channels'], 1)
    return S


def vq_encoder_params(seed=0, cfg=VQ_F4) -> Dict[str, torch.Tensor]:
    """Recipe weights under the fixtures' naming ('vq.' + state_dict name)."""
    return {k: recipe_tensor('vq.' + k, sh, seed) for k, sh in vq_encoder_shapes(cfg).items()}


def vq_encode(P: Dict[str, torch.Tensor], x: torch.Tensor, cfg=VQ_F4) -> torch.Tensor:
    """autoencoder.py:313-316: quant_conv(Encoder(x)) (no quantisation on encode)."""
    def gn(h, pre):
        return F.group_norm(h, 32, P[pre + 'weight'], P[pre + 'bias'], eps=1e-6)

    def swish(h):
        return h * torch.sigmoid(h)

    def conv(h, pre, stride=1, padding=1):
        return F.conv2d(h, P[pre + 'weight'], P[pre + 'bias'], stride=stride, padding=padding)

    def resnet(h, pre):  # model.py:121-141
        y = conv(swish(gn(h, pre + 'norm1.')), pre + 'conv1.')
        y = conv(swish(gn(y, pre + 'norm2.')), pre + 'conv2.')
        if pre + 'nin_shortcut.weight' in P:
            h = conv(h, pre + 'nin_shortcut.', padding=0)
        return h + y

    def attn(h, pre):  # model.py:178-200
        hn = gn(h, pre + 'norm.')
        q, k, v = (conv(hn, pre + n + '.', padding=0) for n in ('q', 'k', 'v'))
        b, c, hh, ww = q.shape
        w_ = torch.bmm(q.reshape(b, c, hh * ww).permute(0, 2, 1), k.reshape(b, c, hh * ww)) * (int(c) ** (-0.5))
        w_ = torch.softmax(w_, dim=2)
        o = torch.bmm(v.reshape(b, c, hh * ww), w_.permute(0, 2, 1)).reshape(b, c, hh, ww)
        return h + conv(o, pre + 'proj_out.', padding=0)

    mult = tuple(cfg['ch_mult'])
    h = conv(x, 'encoder.conv_in.')
    for i in range(len(mult)):  # model.py:434-450
        for j in range(cfg['num_res_blocks']):
            h = resnet(h, f'encoder.down.{i}.block.{j}.')
            if f'encoder.down.{i}.attn.{j}.norm.weight' in P:
                h = attn(h, f'encoder.down.{i}.attn.{j}.')
        if i != len(mult) - 1:  # Downsample(with_conv): pad (0,1,0,1), conv k3 s2 p0 (model.py:72-76)
            h = conv(F.pad(h, (0, 1, 0, 1), mode='constant', value=0), f'encoder.down.{i}.downsample.conv.',
                     stride=2, padding=0)
    h = resnet(h, 'encoder.mid.block_1.')
    h = attn(h, 'encoder.mid.attn_1.')
    h = resnet(h, 'encoder.mid.block_2.')
    h = conv(swish(gn(h, 'encoder.norm_out.')), 'encoder.conv_out.')
    return conv(h, 'quant_conv.', padding=0)


# ----------------------------------------------------------------------------
# Full training step restatement (used as the CPU baseline and as the checker
# of the end-to-end step): q_sample -> UNet -> L1 loss -> backward -> AdamW -> EMA.
# ----------------------------------------------------------------------------

def images_to_input(images_u8: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """Training input of one batch: Shapes3D uint8 HWC images
    (disdata.py:45-97) -> transforms.ToTensor() (x / 255, CHW) -> Normalize((0.5,)*3,
    (0.5,)*3) ((x - 0.5) / 0.5) -> .permute(1, 2, 0) (disdata.py:82-94) -> get_input's
    'b h w c -> b c h w' .float() (ddpm_enc.py:347-353).  torchvision is not installed
    here; ToTensor/Normalize are restated from torchvision's published definitions (the
    reference pins torchvision via encdiff_h100.yaml), so this row is "parity unpinned"
    by reference fixtures."""
    x = images_u8[idx].permute(0, 3, 1, 2).contiguous().to(torch.float32).div(255)
    x = x.sub(0.5).div(0.5)
    return x


class OracleTrainer:
    """CPU restatement of one LatentDiffusion training step (ddpm_enc.py:360-375 ->
    get_input :773-844 (VQ encode * scale_factor), forward :1040-1053, p_losses
    :1183-1253, AdamW :1598-1639, EMA :399-401 -> ema.py:25-44).  ``step`` takes latents
    x0 (the frozen VQ encode skipped); ``step_images`` runs the VQ encode of the images
    first, as the reference's get_input does.  Encoder4 is included (training-mode BN)."""

    def __init__(self, plan: Plan, seed=0, lr=4 * 2e-6, dtype=torch.float32, vq=False, image_size=64):
        self.plan = plan
        shapes = param_shapes(plan)
        self.P = {k: v.to(dtype).requires_grad_(True) for k, v in recipe_params(shapes, seed).items()}
        self.lu = plan.cfg['latent_unit']
        E = encoder4_params(seed, latent_unit=self.lu, context_dim=plan.cfg['context_dim'], image_size=image_size)
        self.E = {k: (v.to(dtype).requires_grad_(True) if v.is_floating_point() and 'running' not in k else v)
                  for k, v in E.items()}
        self.V = {k: v.to(dtype) for k, v in vq_encoder_params(seed).items()} if vq else None
        self.sched = sched_fp32(register_schedule())
        params = list(self.P.values()) + [v for v in self.E.values() if isinstance(v, torch.Tensor)
                                          and v.requires_grad]
        self.opt = torch.optim.AdamW(params, lr=lr)
        self.ema = {k: v.detach().clone() for k, v in self.P.items()}
        self.num_updates = 0
        self.scale_factor = 1.0
        self.last = {}

    def load_state(self, unet, cond, exp_avg, exp_avg_sq, step, ema, num_updates):
        """Start from a given training state (e.g. the HIP trainer's after its warm-up):
        parameters, AdamW moments (keyed by parameter name, 'cond.' prefix for Encoder4),
        the AdamW step count, the EMA shadow and LitEma.num_updates."""
        with torch.no_grad():
            for k, p in self.P.items():
                p.copy_(unet[k])
            for k, p in self.E.items():
                if k in cond and isinstance(p, torch.Tensor):
                    p.copy_(cond[k])
        for name, p in list(self.P.items()) + [('cond.' + k, v) for k, v in self.E.items()]:
            if isinstance(p, torch.Tensor) and p.requires_grad:
                self.opt.state[p] = {'step': torch.tensor(float(step)), 'exp_avg': exp_avg[name].clone(),
                                     'exp_avg_sq': exp_avg_sq[name].clone()}
        self.ema = {k: v.detach().clone() for k, v in ema.items()}
        self.num_updates = int(num_updates)

    def step(self, x0, img, t, noise, seed=None):
        """One step; ``seed``: an upstream gradient for the model output to backpropagate
        instead of d loss / d eps (the L1 seed sign(eps - noise)/N is discontinuous, so a
        checker shares the seed the device computed)."""
        self.opt.zero_grad(set_to_none=True)
        c = encoder4_forward(self.E, img, latent_unit=self.lu)
        x_noisy = q_sample(self.sched, x0, t, noise)
        out = unet_forward(self.P, self.plan, x_noisy, t, [c])
        loss, ld = p_losses_from_output(self.sched, out, noise, t)
        if seed is None:
            loss.backward()
        else:
            out.backward(seed)
        self.opt.step()
        with torch.no_grad():
            self.ema, self.num_updates = ema_update(self.ema, {k: v.detach() for k, v in self.P.items()},
                                                    self.num_updates)
        self.last = dict(eps=out.detach(), x0=x0, loss=loss.detach())
        return loss.detach()

    def encode_images(self, img):
        """get_input (ddpm_enc.py:780-784): z = scale_factor * VQ.encode(img), no grad."""
        with torch.no_grad():
            return self.scale_factor * vq_encode(self.V, img)

    def step_images(self, img, t, noise, seed=None):
        return self.step(self.encode_images(img), img, t, noise, seed=seed)
