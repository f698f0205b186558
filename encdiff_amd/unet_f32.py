"""The denoiser forward at the reference's precision (fp32 activations end to end).

SURVEY §8(b) convention (5): an fp32 path through the C-ABI for parity.  The reference computes
in fp32 (main_val.py:525); the product step runs bf16 activations (unet.py).  This executor
restates openaimodel_enc.UNetModel.forward (openaimodel_enc.py:712-748) -- ResBlock._forward
(:255-275), SpatialTransformer / BasicTransformerBlock / CrossAttention / GEGLU
(attention.py:37-261), timestep_embedding (util.py:179-199), GroupNorm32 (util.py:242-244) --
on the SAME entry points with ``dtype = ENCDIFF_DT_F32`` (fp32.hip): MFMA f32 GEMMs with implicit
im2col, two-pass GroupNorm / LayerNorm, exact-softmax attention, fp32 elementwise.  Weights are
the fp32 master arena itself (conv weights stored channels-last are the GEMM's [cout][9*cin]
operand as they are).  Forward only, no saved activations: the parity / reference-precision
sampling path (UNetModel.forward with ``hip_precision = "fp32"``), held to 1e-4 rel-L2 against
the reference's own output (tests/test_gpu_fp32.py).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

from . import _lib as L
from . import ops
from .ops import Geom

F32 = torch.float32
GN_EPS, ST_GN_EPS, LN_EPS = 1e-5, 1e-6, 1e-5


class UNetF32:
    def __init__(self, ex):
        """ex: the model's UNetExecutor (its spec, arena and grouped-weight spans)."""
        self.ex = ex
        self.spec, self.arena = ex.spec, ex.arena
        self.dev = ex.dev
        self._prep: Dict[str, Tuple[int, int, torch.Tensor]] = {}

    # ------------------------------------------------------------ weights
    def P(self, name):
        return self.arena.f32(name)

    def lin_w(self, name):
        w = self.P(name)
        return w.reshape(w.shape[0], -1)

    def conv_w(self, name, cpad=None):
        """[cout][9 * cin] fp32, tap-major with the channel inner (the im2col order).  Arena
        channels-last weights are that already; reference-layout ones are re-laid once per
        parameter version (cpad: channels zero-padded to cpad)."""
        a = self.arena
        if name in a.cl and cpad is None:
            return a.raw(a.master, name)
        key = (a.master._version, a.gen)
        hit = self._prep.get(name)
        if hit is None or hit[0] != key:
            w = self.P(name)
            co, ci = w.shape[0], w.shape[1]
            cp = cpad or ci
            out = torch.zeros(co, 3, 3, cp, device=self.dev, dtype=F32)
            out[..., :ci] = w.detach().permute(0, 2, 3, 1)
            hit = self._prep[name] = (key, 0, out.reshape(co, 9 * cp))
        return hit[2]

    def span(self, names):
        o, n = self.arena.span(names)
        return self.arena.master[o:o + n]

    def _t(self, rows, cols):
        return torch.empty(rows, cols, device=self.dev, dtype=F32)

    # ------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, x, t, ctx):
        """x (B, C, H, W) fp32, t (B,) int64, ctx (B, latent_unit * context_dim) fp32 -> eps."""
        sp, ex = self.spec, self.ex
        B, cin0, H, W = x.shape
        mc = ex.mc
        g0 = Geom(B, H, W)
        x = x.float().contiguous()
        t = t.long().contiguous()
        # time embedding MLP (openaimodel_enc.py:726-727) and every ResBlock's emb_layers
        temb = self._t(B, mc)
        ops.timestep_embedding_f32(t, mc, temb)
        h1 = self._t(B, 4 * mc)
        ops.linear_f32(temb, self.lin_w("time_embed.0.weight"), h1, bias=self.P("time_embed.0.bias"))
        ops.ew_f32(L.EW_SILU, h1, h1)
        emb = self._t(B, 4 * mc)
        ops.linear_f32(h1, self.lin_w("time_embed.2.weight"), emb, bias=self.P("time_embed.2.bias"))
        ops.ew_f32(L.EW_SILU, emb, emb)
        E = self._t(B, sp.film_total)
        emb_w = self.span([r.prefix + "emb_layers.1.weight" for r in sp.res]).view(sp.film_total, 4 * mc)
        ops.linear_f32(emb, emb_w, E, bias=self.span(ex.emb_bias_names))
        # every cross-attention's K / V of the concept tokens
        ctx2 = ctx.float().contiguous().view(B * ex.lu, ex.cd)
        kv_names = []
        for s in sp.sts:
            tb = s.prefix + "transformer_blocks.0.attn2."
            kv_names += [tb + "to_k.weight", tb + "to_v.weight"]
        KV = self._t(B * ex.lu, sp.kv_total)
        ops.linear_f32(ctx2, self.span(kv_names).view(sp.kv_total, ex.cd), KV)
        self.E, self.KV = E, KV
        # input conv over channel-padded rows
        x8 = self._t(B * H * W, 8)
        ops.nchw_rows_f32(x, B, cin0, H * W, 8, x8, 8, to_rows=True)
        h = self._t(B * H * W, mc)
        ops.conv3x3_f32(x8, g0, 8, self.conv_w("input_blocks.0.0.weight", cpad=8), h,
                        bias=self.P("input_blocks.0.0.bias"))
        hs = [h]
        for blk in sp.input_blocks[1:]:
            for layer in blk:
                h = self._layer(layer, h)
            hs.append(h)
        for layer in sp.middle:
            h = self._layer(layer, h)
        for blk in sp.output_blocks:
            skip = hs.pop()
            c1, c2 = h.shape[1], skip.shape[1]
            cat = self._t(h.shape[0], c1 + c2)  # torch.cat([h, hs.pop()], 1) (openaimodel_enc.py:740)
            ops.ew_f32(L.EW_COPY, h, cat[:, :c1])
            ops.ew_f32(L.EW_COPY, skip, cat[:, c1:])
            h = cat
            for layer in blk:
                h = self._layer(layer, h)
        # out: GroupNorm32 + SiLU + conv3x3 (openaimodel_enc.py:684-688)
        a = self._t(h.shape[0], h.shape[1])
        ops.groupnorm_f32(h, g0, self.P("out.0.weight"), self.P("out.0.bias"), a, self._stats(B), GN_EPS, True)
        co = self.P("out.2.weight").shape[0]
        rows = self._t(B * H * W, co)
        ops.conv3x3_f32(a, g0, h.shape[1], self.conv_w("out.2.weight"), rows, bias=self.P("out.2.bias"))
        eps = torch.empty(B, co, H, W, device=self.dev, dtype=F32)
        ops.nchw_rows_f32(rows, B, co, H * W, co, eps, co, to_rows=False)
        return eps

    def _stats(self, B):
        return torch.empty(B * 64, device=self.dev, dtype=F32)

    def _layer(self, layer, x):
        from .unet import ResSpec
        return self._res(layer, x) if isinstance(layer, ResSpec) else self._st(layer, x)

    def _res(self, r, x):
        """openaimodel_enc.py:255-275, use_scale_shift_norm, resblock_updown."""
        B = x.shape[0] // (r.hin * r.hin)
        gi, go = Geom(B, r.hin, r.hin), Geom(B, r.hout, r.hout)
        p = r.prefix
        a1 = self._t(x.shape[0], r.cin)
        ops.groupnorm_f32(x, gi, self.P(p + "in_layers.0.weight"), self.P(p + "in_layers.0.bias"), a1,
                          self._stats(B), GN_EPS, True)
        rs = L.RESAMPLE_NONE
        xs = x
        if r.updown == L.RESAMPLE_DOWN2:  # h_upd / x_upd = AvgPool2d(2) before the in_conv (:256-261)
            a1d = self._t(go.pixels, r.cin)
            ops.ew_f32(L.EW_RESAMPLE, a1, a1d, resample=L.RESAMPLE_DOWN2, g=go)
            a1 = a1d
            xs = self._t(go.pixels, r.cin)
            ops.ew_f32(L.EW_RESAMPLE, x, xs, resample=L.RESAMPLE_DOWN2, g=go)
        elif r.updown == L.RESAMPLE_UP2:  # nearest x2: read through the conv's gather; x upsampled
            rs = L.RESAMPLE_UP2
            xs = self._t(go.pixels, r.cin)
            ops.ew_f32(L.EW_RESAMPLE, x, xs, resample=L.RESAMPLE_UP2, g=go)
        h1 = self._t(go.pixels, r.cout)
        ops.conv3x3_f32(a1, go, r.cin, self.conv_w(p + "in_layers.2.weight"), h1, bias=self.P(p + "in_layers.2.bias"),
                        resample=rs)
        a2 = self._t(go.pixels, r.cout)
        ops.groupnorm_f32(h1, go, self.P(p + "out_layers.0.weight"), self.P(p + "out_layers.0.bias"), a2,
                          self._stats(B), GN_EPS, True, film=self.E[:, r.film_off:], ld_film=self.E.shape[1])
        out = self._t(go.pixels, r.cout)
        if r.cin != r.cout:
            ops.linear_f32(xs, self.lin_w(p + "skip_connection.weight"), out, bias=self.P(p + "skip_connection.bias"))
            resid = out
        else:
            resid = xs
        ops.conv3x3_f32(a2, go, r.cout, self.conv_w(p + "out_layers.3.weight"), out,
                        bias=self.P(p + "out_layers.3.bias"), resid=resid)
        return out

    def _st(self, s, x):
        """attention.py:250-261 with BasicTransformerBlock :211-215 (depth 1)."""
        c, ntok = s.c, s.h * s.h
        M = x.shape[0]
        B = M // ntok
        p, tb = s.prefix, s.prefix + "transformer_blocks.0."
        g = Geom(B, s.h, s.h)
        gn = self._t(M, c)
        ops.groupnorm_f32(x, g, self.P(p + "norm.weight"), self.P(p + "norm.bias"), gn, self._stats(B), ST_GN_EPS, False)
        t0 = self._t(M, c)
        ops.linear_f32(gn, self.lin_w(p + "proj_in.weight"), t0, bias=self.P(p + "proj_in.bias"))
        # attn1 (self)
        n = self._t(M, c)
        ops.layernorm_f32(t0, self.P(tb + "norm1.weight"), self.P(tb + "norm1.bias"), n, LN_EPS)
        qkv = self._t(M, 3 * c)
        ops.linear_f32(n, self.span([tb + "attn1.to_q.weight", tb + "attn1.to_k.weight",
                                     tb + "attn1.to_v.weight"]).view(3 * c, c), qkv)
        o = self._t(M, c)
        ops.attention_f32(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], o, B, s.heads, ntok, ntok, s.dh)
        t1 = self._t(M, c)
        ops.linear_f32(o, self.lin_w(tb + "attn1.to_out.0.weight"), t1, bias=self.P(tb + "attn1.to_out.0.bias"),
                       resid=t0)
        # attn2 (cross, to the concept tokens)
        ops.layernorm_f32(t1, self.P(tb + "norm2.weight"), self.P(tb + "norm2.bias"), n, LN_EPS)
        q2 = self._t(M, c)
        ops.linear_f32(n, self.lin_w(tb + "attn2.to_q.weight"), q2)
        lu = self.ex.lu
        ops.attention_f32(q2, self.KV[:, s.kv_off:s.kv_off + c], self.KV[:, s.kv_off + c:s.kv_off + 2 * c], o,
                          B, s.heads, ntok, lu, s.dh)
        t2 = self._t(M, c)
        ops.linear_f32(o, self.lin_w(tb + "attn2.to_out.0.weight"), t2, bias=self.P(tb + "attn2.to_out.0.bias"),
                       resid=t1)
        # GEGLU feed-forward
        ops.layernorm_f32(t2, self.P(tb + "norm3.weight"), self.P(tb + "norm3.bias"), n, LN_EPS)
        f = self._t(M, 8 * c)
        ops.linear_f32(n, self.lin_w(tb + "ff.net.0.proj.weight"), f, bias=self.P(tb + "ff.net.0.proj.bias"))
        a = self._t(M, 4 * c)
        ops.ew_f32(L.EW_GEGLU, f, a, cols=4 * c)
        t3 = self._t(M, c)
        ops.linear_f32(a, self.lin_w(tb + "ff.net.2.weight"), t3, bias=self.P(tb + "ff.net.2.bias"), resid=t2)
        out = self._t(M, c)
        ops.linear_f32(t3, self.lin_w(p + "proj_out.weight"), out, bias=self.P(p + "proj_out.bias"), resid=x)
        return out
