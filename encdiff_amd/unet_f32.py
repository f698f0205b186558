"""The denoiser at the reference's precision (fp32 activations end to end), forward AND backward.

SURVEY §8(b) convention (5): an fp32 path through the C-ABI for parity.  The reference computes
in fp32 (main_val.py:525); the product step runs bf16 activations (unet.py).  This executor
restates openaimodel_enc.UNetModel.forward (openaimodel_enc.py:712-748) -- ResBlock._forward
(:255-275), SpatialTransformer / BasicTransformerBlock / CrossAttention / GEGLU
(attention.py:37-261), timestep_embedding (util.py:179-199), GroupNorm32 (util.py:242-244) --
and its autograd backward on the SAME entry points with ``dtype = ENCDIFF_DT_F32`` (fp32.hip):
MFMA f32 GEMMs with implicit im2col in every operand form (forward, input gradient through the
flipped kernel, weight gradient over im2col columns), two-pass GroupNorm / LayerNorm and their
backward from the saved statistics, exact-softmax attention and its backward from the saved
log-sum-exp, fp32 elementwise (SiLU, GEGLU, resample and their adjoints).  Weights are the fp32
master arena itself (conv weights stored channels-last are the GEMM's [cout][9*cin] operand as
they are); weight gradients accumulate into the arena's gradient buffer in the same layout, the
GroupNorm / LayerNorm affine gradients through per-image / per-part partial sums
(encdiff_reduce_partials).

UNetModel with ``hip_precision = "fp32"`` runs it: under no_grad the forward alone (parity /
reference-precision sampling), with grad the forward saves its activations and the autograd
function's backward returns d x_t and d context and fills every UNet parameter gradient
(tests/test_gpu_fp32.py holds them to 1e-4 rel-L2 against the reference's own fp32 gradients).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

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
        self.saved = None

    # ------------------------------------------------------------ weights / gradients
    def P(self, name):
        return self.arena.f32(name)

    def lin_w(self, name):
        w = self.P(name)
        return w.reshape(w.shape[0], -1)

    def conv_w(self, name, cpad=None, rows=None):
        """[cout][9 * cin] fp32, tap-major with the channel inner (the im2col order).  Arena
        channels-last weights are that already; reference-layout ones are re-laid once per
        parameter version (cpad: channels zero-padded to cpad; rows: output rows zero-padded)."""
        a = self.arena
        if name in a.cl and cpad is None and rows is None:
            return a.raw(a.master, name)
        key = (a.master._version, a.gen, cpad, rows)
        hit = self._prep.get(name)
        if hit is None or hit[0] != key:
            w = self.P(name)
            co, ci = w.shape[0], w.shape[1]
            cp = cpad or ci
            out = torch.zeros(rows or co, 3, 3, cp, device=self.dev, dtype=F32)
            out[:co, ..., :ci] = w.detach().permute(0, 2, 3, 1)
            hit = self._prep[name] = (key, 0, out.reshape(rows or co, 9 * cp))
        return hit[2]

    def span(self, names):
        o, n = self.arena.span(names)
        return self.arena.master[o:o + n]

    def G(self, name):
        """The arena gradient of `name` in storage order: [rows][cols] for matrices / conv weights
        (channels-last convs: [co][9*ci]), flat for vectors."""
        a = self.arena
        o, shp = a.offsets[name]
        if len(shp) == 1:
            return a.grad[o:o + shp[0]]
        return a.raw(a.grad, name)

    def Gspan(self, names, rows=None):
        o, n = self.arena.span(names)
        g = self.arena.grad[o:o + n]
        return g if rows is None else g.view(rows, n // rows)

    def _t(self, rows, cols, zero=False):
        f = torch.zeros if zero else torch.empty
        return f(rows, cols, device=self.dev, dtype=F32)

    def _affine(self, parts, rows, gamma_name, beta_name):
        """Fold per-image / per-part affine partial sums [rows][2][c] into the arena gradients."""
        a = self.arena
        c = parts.shape[1] // 2
        og, _ = a.offsets[gamma_name]
        ob, _ = a.offsets[beta_name]
        idx = torch.cat([torch.arange(og, og + c), torch.arange(ob, ob + c)]).to(device=self.dev, dtype=torch.int32)
        ops.reduce_partials(parts, parts.stride(0), rows, 2 * c, idx, a.grad)

    # ------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, x, t, ctx, save=False):
        """x (B, C, H, W) fp32, t (B,) int64, ctx (B, latent_unit * context_dim) fp32 -> eps.
        save: keep every activation the backward reads (self.saved)."""
        sp, ex = self.spec, self.ex
        B, cin0, H, W = x.shape
        mc = ex.mc
        g0 = Geom(B, H, W)
        x = x.float().contiguous()
        t = t.long().contiguous()
        S: Dict[str, object] = {"B": B, "H": H, "cin0": cin0} if save else None
        self.S = S
        # time embedding MLP (openaimodel_enc.py:726-727) and every ResBlock's emb_layers
        temb = self._t(B, mc)
        ops.timestep_embedding_f32(t, mc, temb)
        h1 = self._t(B, 4 * mc)
        ops.linear_f32(temb, self.lin_w("time_embed.0.weight"), h1, bias=self.P("time_embed.0.bias"))
        h1a = self._t(B, 4 * mc)
        ops.ew_f32(L.EW_SILU, h1, h1a)
        embp = self._t(B, 4 * mc)
        ops.linear_f32(h1a, self.lin_w("time_embed.2.weight"), embp, bias=self.P("time_embed.2.bias"))
        emb = self._t(B, 4 * mc)
        ops.ew_f32(L.EW_SILU, embp, emb)
        E = self._t(B, sp.film_total)
        emb_w = self.span([r.prefix + "emb_layers.1.weight" for r in sp.res]).view(sp.film_total, 4 * mc)
        ops.linear_f32(emb, emb_w, E, bias=self.span(ex.emb_bias_names))
        # every cross-attention's K / V of the concept tokens
        ctx2 = ctx.float().contiguous().view(B * ex.lu, ex.cd)
        KV = self._t(B * ex.lu, sp.kv_total)
        ops.linear_f32(ctx2, self.span(self._kv_names()).view(sp.kv_total, ex.cd), KV)
        self.E, self.KV = E, KV
        if save:
            S.update(temb=temb, h1=h1, h1a=h1a, embp=embp, emb=emb, ctx2=ctx2)
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
        if save:
            S.update(x8=x8, hs_c=[t_.shape[1] for t_ in hs])
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
        st = self._stats(B)
        ops.groupnorm_f32(h, g0, self.P("out.0.weight"), self.P("out.0.bias"), a, st, GN_EPS, True)
        co = self.P("out.2.weight").shape[0]
        rows = self._t(B * H * W, co)
        ops.conv3x3_f32(a, g0, h.shape[1], self.conv_w("out.2.weight"), rows, bias=self.P("out.2.bias"))
        eps = torch.empty(B, co, H, W, device=self.dev, dtype=F32)
        ops.nchw_rows_f32(rows, B, co, H * W, co, eps, co, to_rows=False)
        if save:
            S.update(h_last=h, a_out=a, st_out=st)
            self.saved = S
        return eps

    def _kv_names(self):
        names = []
        for s in self.spec.sts:
            tb = s.prefix + "transformer_blocks.0.attn2."
            names += [tb + "to_k.weight", tb + "to_v.weight"]
        return names

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
        st1 = self._stats(B)
        ops.groupnorm_f32(x, gi, self.P(p + "in_layers.0.weight"), self.P(p + "in_layers.0.bias"), a1, st1, GN_EPS,
                          True)
        rs = L.RESAMPLE_NONE
        xs = x
        a1c = a1  # the conv's source rows (resampled on the fly for UP2)
        if r.updown == L.RESAMPLE_DOWN2:  # h_upd / x_upd = AvgPool2d(2) before the in_conv (:256-261)
            a1c = self._t(go.pixels, r.cin)
            ops.ew_f32(L.EW_RESAMPLE, a1, a1c, resample=L.RESAMPLE_DOWN2, g=go)
            xs = self._t(go.pixels, r.cin)
            ops.ew_f32(L.EW_RESAMPLE, x, xs, resample=L.RESAMPLE_DOWN2, g=go)
        elif r.updown == L.RESAMPLE_UP2:  # nearest x2: read through the conv's gather; x upsampled
            rs = L.RESAMPLE_UP2
            xs = self._t(go.pixels, r.cin)
            ops.ew_f32(L.EW_RESAMPLE, x, xs, resample=L.RESAMPLE_UP2, g=go)
        h1 = self._t(go.pixels, r.cout)
        ops.conv3x3_f32(a1c, go, r.cin, self.conv_w(p + "in_layers.2.weight"), h1, bias=self.P(p + "in_layers.2.bias"),
                        resample=rs)
        a2 = self._t(go.pixels, r.cout)
        st2 = self._stats(B)
        ops.groupnorm_f32(h1, go, self.P(p + "out_layers.0.weight"), self.P(p + "out_layers.0.bias"), a2, st2, GN_EPS,
                          True, film=self.E[:, r.film_off:], ld_film=self.E.shape[1])
        out = self._t(go.pixels, r.cout)
        if r.cin != r.cout:
            ops.linear_f32(xs, self.lin_w(p + "skip_connection.weight"), out, bias=self.P(p + "skip_connection.bias"))
            resid = out
        else:
            resid = xs
        ops.conv3x3_f32(a2, go, r.cout, self.conv_w(p + "out_layers.3.weight"), out,
                        bias=self.P(p + "out_layers.3.bias"), resid=resid)
        if self.S is not None:
            self.S[p] = dict(x=x, st1=st1, a1c=a1c, rs=rs, xs=xs, h1=h1, a2=a2, st2=st2)
        return out

    def _st(self, s, x):
        """attention.py:250-261 with BasicTransformerBlock :211-215 (depth 1)."""
        c, ntok = s.c, s.h * s.h
        M = x.shape[0]
        B = M // ntok
        p, tb = s.prefix, s.prefix + "transformer_blocks.0."
        g = Geom(B, s.h, s.h)
        save = self.S is not None
        gn = self._t(M, c)
        stg = self._stats(B)
        ops.groupnorm_f32(x, g, self.P(p + "norm.weight"), self.P(p + "norm.bias"), gn, stg, ST_GN_EPS, False)
        t0 = self._t(M, c)
        ops.linear_f32(gn, self.lin_w(p + "proj_in.weight"), t0, bias=self.P(p + "proj_in.bias"))
        lstat = [torch.empty(M * 2, device=self.dev, dtype=F32) if save else None for _ in range(3)]
        lse = [torch.empty(B * s.heads * ntok, device=self.dev, dtype=F32) if save else None for _ in range(2)]
        # attn1 (self)
        n1 = self._t(M, c)
        ops.layernorm_f32(t0, self.P(tb + "norm1.weight"), self.P(tb + "norm1.bias"), n1, LN_EPS, stats=lstat[0])
        qkv = self._t(M, 3 * c)
        ops.linear_f32(n1, self.span([tb + "attn1.to_q.weight", tb + "attn1.to_k.weight",
                                      tb + "attn1.to_v.weight"]).view(3 * c, c), qkv)
        o1 = self._t(M, c)
        ops.attention_f32(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], o1, B, s.heads, ntok, ntok, s.dh, lse=lse[0])
        t1 = self._t(M, c)
        ops.linear_f32(o1, self.lin_w(tb + "attn1.to_out.0.weight"), t1, bias=self.P(tb + "attn1.to_out.0.bias"),
                       resid=t0)
        # attn2 (cross, to the concept tokens)
        n2 = self._t(M, c) if save else n1
        ops.layernorm_f32(t1, self.P(tb + "norm2.weight"), self.P(tb + "norm2.bias"), n2, LN_EPS, stats=lstat[1])
        q2 = self._t(M, c)
        ops.linear_f32(n2, self.lin_w(tb + "attn2.to_q.weight"), q2)
        lu = self.ex.lu
        o2 = self._t(M, c) if save else o1
        ops.attention_f32(q2, self.KV[:, s.kv_off:s.kv_off + c], self.KV[:, s.kv_off + c:s.kv_off + 2 * c], o2,
                          B, s.heads, ntok, lu, s.dh, lse=lse[1])
        t2 = self._t(M, c)
        ops.linear_f32(o2, self.lin_w(tb + "attn2.to_out.0.weight"), t2, bias=self.P(tb + "attn2.to_out.0.bias"),
                       resid=t1)
        # GEGLU feed-forward
        n3 = self._t(M, c) if save else n1
        ops.layernorm_f32(t2, self.P(tb + "norm3.weight"), self.P(tb + "norm3.bias"), n3, LN_EPS, stats=lstat[2])
        f = self._t(M, 8 * c)
        ops.linear_f32(n3, self.lin_w(tb + "ff.net.0.proj.weight"), f, bias=self.P(tb + "ff.net.0.proj.bias"))
        a = self._t(M, 4 * c)
        ops.ew_f32(L.EW_GEGLU, f, a, cols=4 * c)
        t3 = self._t(M, c)
        ops.linear_f32(a, self.lin_w(tb + "ff.net.2.weight"), t3, bias=self.P(tb + "ff.net.2.bias"), resid=t2)
        out = self._t(M, c)
        ops.linear_f32(t3, self.lin_w(p + "proj_out.weight"), out, bias=self.P(p + "proj_out.bias"), resid=x)
        if save:
            self.S[p] = dict(x=x, stg=stg, gn=gn, t0=t0, n1=n1, qkv=qkv, o1=o1, t1=t1, n2=n2, q2=q2, o2=o2, t2=t2,
                             n3=n3, f=f, a=a, t3=t3, lstat=lstat, lse=lse)
        return out

    # ------------------------------------------------------------ backward
    @torch.no_grad()
    def backward(self, d_eps) -> Tuple[torch.Tensor, torch.Tensor]:
        """d_eps (B, C, H, W) -> (d x_t (B, C, H, W), d context (B, latent_unit * context_dim)); every
        UNet weight gradient is ADDED to the arena's gradient buffer (the caller zeroes it)."""
        S = self.saved
        assert S is not None, "backward() follows forward(save=True)"
        sp, ex = self.spec, self.ex
        B, H, cin0 = S["B"], S["H"], S["cin0"]
        mc = ex.mc
        g0 = Geom(B, H, H)
        self.dE = self._t(B, sp.film_total, zero=True)
        self.dKV = self._t(B * ex.lu, sp.kv_total, zero=True)
        # out conv (mc -> 3), output rows padded to 4 channels
        co = sp.cfg["out_channels"]
        d4 = self._t(g0.pixels, 4)
        ops.nchw_rows_f32(d_eps.float().contiguous(), B, co, H * H, 4, d4, 4, to_rows=True)
        a_out = S["a_out"]
        c_last = a_out.shape[1]
        d_aout = self._t(g0.pixels, c_last)
        ops.conv3x3_dgrad_f32(d4, g0, self.conv_w("out.2.weight", rows=4), d_aout)
        dw4 = self._t(4, 9 * c_last, zero=True)
        db4 = torch.zeros(4, device=self.dev, dtype=F32)
        ops.conv3x3_wgrad_f32(d4, a_out, g0, c_last, dw4, db=db4)
        ops.grad_fold(dw4, co, c_last, c_last, 9, self.arena.grad_of("out.2.weight"), db4, self.G("out.2.bias"))
        dh = self._t(g0.pixels, c_last)
        self._gn_bwd(S["h_last"], g0, "out.0.", S["st_out"], True, d_aout, dh, accumulate=False)
        # output blocks, middle block, input blocks (reverse order); g_hs[i]: gradient of hs[i]
        nhs = len(sp.input_blocks)
        g_hs: List[torch.Tensor] = [None] * nhs
        dout = dh
        for j in range(len(sp.output_blocks) - 1, -1, -1):
            blk = sp.output_blocks[j]
            for li in range(len(blk) - 1, -1, -1):
                dout = self._layer_bwd(blk[li], dout)
            i = nhs - 1 - j
            c2 = S["hs_c"][i]
            c1 = dout.shape[1] - c2
            g_hs[i] = dout[:, c1:].contiguous()
            dout = dout[:, :c1].contiguous()
        for li in range(len(sp.middle) - 1, -1, -1):
            dout = self._layer_bwd(sp.middle[li], dout)
        ops.ew_f32(L.EW_ADD, g_hs[nhs - 1], g_hs[nhs - 1], x2=dout)
        for i in range(nhs - 1, 0, -1):
            dout = g_hs[i]
            for layer in reversed(sp.input_blocks[i]):
                dout = self._layer_bwd(layer, dout)
            ops.ew_f32(L.EW_ADD, g_hs[i - 1], g_hs[i - 1], x2=dout)
        # input conv (3 -> mc over channel-padded rows): weight gradient and d x_t
        dy0 = g_hs[0]
        dwi = self._t(mc, 72, zero=True)
        ops.conv3x3_wgrad_f32(dy0, S["x8"], g0, 8, dwi, db=self.G("input_blocks.0.0.bias"))
        ops.grad_fold(dwi, mc, cin0, 8, 9, self.arena.grad_of("input_blocks.0.0.weight"))
        dx8 = self._t(g0.pixels, 8)
        ops.conv3x3_dgrad_f32(dy0, g0, self.conv_w("input_blocks.0.0.weight", cpad=8), dx8)
        dx = torch.empty(B, cin0, H, H, device=self.dev, dtype=F32)
        ops.nchw_rows_f32(dx8, B, cin0, H * H, 8, dx, 8, to_rows=False)
        # batched emb_layers -> time MLP (openaimodel_enc.py:507-512, 218-224)
        emb_names = [r.prefix + "emb_layers.1.weight" for r in sp.res]
        emb_w = self.span(emb_names).view(sp.film_total, 4 * mc)
        d_emb = self._t(B, 4 * mc)
        ops.linear_dgrad_f32(self.dE, emb_w, d_emb)
        bo, bn = self.arena.span(ex.emb_bias_names)
        ops.linear_wgrad_f32(self.dE, S["emb"], self.Gspan(emb_names, sp.film_total), db=self.arena.grad[bo:bo + bn])
        d_embp = self._t(B, 4 * mc)
        ops.ew_f32(L.EW_SILU_BWD, S["embp"], d_embp, x2=d_emb)
        ops.linear_wgrad_f32(d_embp, S["h1a"], self.G("time_embed.2.weight"), db=self.G("time_embed.2.bias"))
        d_h1a = self._t(B, 4 * mc)
        ops.linear_dgrad_f32(d_embp, self.lin_w("time_embed.2.weight"), d_h1a)
        d_h1 = self._t(B, 4 * mc)
        ops.ew_f32(L.EW_SILU_BWD, S["h1"], d_h1, x2=d_h1a)
        ops.linear_wgrad_f32(d_h1, S["temb"], self.G("time_embed.0.weight"), db=self.G("time_embed.0.bias"))
        # every cross-attention K / V projection -> d context
        kv_names = self._kv_names()
        d_ctx2 = self._t(B * ex.lu, ex.cd)
        ops.linear_dgrad_f32(self.dKV, self.span(kv_names).view(sp.kv_total, ex.cd), d_ctx2)
        ops.linear_wgrad_f32(self.dKV, S["ctx2"], self.Gspan(kv_names, sp.kv_total))
        self.saved = None
        return dx, d_ctx2.view(B, ex.lu * ex.cd)

    def _gn_bwd(self, x, g, prefix, stats, silu, dy, dx, accumulate, film=None, resid=None, eps_st=False):
        c = x.shape[1]
        parts = self._t(g.batch, 2 * c)
        kw = {}
        if film is not None:
            kw = dict(film=self.E[:, film:], ld_film=self.E.shape[1], dfilm=self.dE[:, film:], ld_dfilm=self.dE.shape[1])
        ops.groupnorm_bwd_f32(x, g, self.P(prefix + "weight"), self.P(prefix + "bias"), stats, silu, dy, dx,
                              parts[:, :c], parts[:, c:], parts.stride(0), accumulate=accumulate, resid=resid, **kw)
        self._affine(parts, g.batch, prefix + "weight", prefix + "bias")

    def _ln_bwd(self, x, prefix, stats, dy, dx, resid):
        rows, c = x.shape
        nparts = min(64, rows)
        parts = self._t(nparts, 2 * c)
        ops.layernorm_bwd_f32(x, self.P(prefix + "weight"), stats, dy, dx, parts[:, :c], parts[:, c:], nparts,
                              parts.stride(0), resid=resid)
        self._affine(parts, nparts, prefix + "weight", prefix + "bias")

    def _lin_bwd(self, name_w, name_b, dy, x, dx=None, w=None, dw=None):
        """y = x W^T (+ b): dW += dy^T x, db += sum dy; dx = dy W (when dx is given)."""
        ops.linear_wgrad_f32(dy, x, self.G(name_w) if dw is None else dw, db=self.G(name_b) if name_b else None)
        if dx is not None:
            ops.linear_dgrad_f32(dy, self.lin_w(name_w) if w is None else w, dx)

    def _layer_bwd(self, layer, dout):
        from .unet import ResSpec
        return self._res_bwd(layer, dout) if isinstance(layer, ResSpec) else self._st_bwd(layer, dout)

    def _res_bwd(self, r, dout):
        St = self.S[r.prefix]
        p = r.prefix
        x = St["x"]
        B = x.shape[0] // (r.hin * r.hin)
        gi, go = Geom(B, r.hin, r.hin), Geom(B, r.hout, r.hout)
        # out_layers.3 (conv2, zero_module in the reference; recipe weights here)
        ops.conv3x3_wgrad_f32(dout, St["a2"], go, r.cout, self.G(p + "out_layers.3.weight"),
                              db=self.G(p + "out_layers.3.bias"))
        d_a2 = self._t(go.pixels, r.cout)
        ops.conv3x3_dgrad_f32(dout, go, self.conv_w(p + "out_layers.3.weight"), d_a2)
        d_h1 = self._t(go.pixels, r.cout)
        self._gn_bwd(St["h1"], go, p + "out_layers.0.", St["st2"], True, d_a2, d_h1, False, film=r.film_off)
        # in_layers.2 (conv1) over the resampled GroupNorm output
        ops.conv3x3_wgrad_f32(d_h1, St["a1c"], go, r.cin, self.G(p + "in_layers.2.weight"),
                              db=self.G(p + "in_layers.2.bias"), resample=St["rs"])
        d_a1c = self._t(go.pixels, r.cin)
        ops.conv3x3_dgrad_f32(d_h1, go, self.conv_w(p + "in_layers.2.weight"), d_a1c)
        if r.updown != L.RESAMPLE_NONE:
            d_a1 = self._t(gi.pixels, r.cin)
            ops.ew_f32(L.EW_RESAMPLE_BWD, d_a1c, d_a1, resample=r.updown, g=gi)
        else:
            d_a1 = d_a1c
        # skip branch: 1x1 conv when the channel count changes, else identity
        if r.cin != r.cout:
            d_xs = self._t(go.pixels, r.cin)
            self._lin_bwd(p + "skip_connection.weight", p + "skip_connection.bias", dout, St["xs"], d_xs)
        else:
            d_xs = dout
        dx = self._t(gi.pixels, r.cin)
        if r.updown != L.RESAMPLE_NONE:
            ops.ew_f32(L.EW_RESAMPLE_BWD, d_xs, dx, resample=r.updown, g=gi)
            self._gn_bwd(x, gi, p + "in_layers.0.", St["st1"], True, d_a1, dx, True)
        else:
            self._gn_bwd(x, gi, p + "in_layers.0.", St["st1"], True, d_a1, dx, False, resid=d_xs)
        return dx

    def _st_bwd(self, s, dout):
        St = self.S[s.prefix]
        c, ntok = s.c, s.h * s.h
        x = St["x"]
        M = x.shape[0]
        B = M // ntok
        p, tb = s.prefix, s.prefix + "transformer_blocks.0."
        lstat, lse = St["lstat"], St["lse"]
        # proj_out (+ x): d t3
        d_t3 = self._t(M, c)
        self._lin_bwd(p + "proj_out.weight", p + "proj_out.bias", dout, St["t3"], d_t3)
        # ff.net.2 (+ t2), GEGLU, ff.net.0.proj, norm3
        d_a = self._t(M, 4 * c)
        self._lin_bwd(tb + "ff.net.2.weight", tb + "ff.net.2.bias", d_t3, St["a"], d_a)
        d_f = self._t(M, 8 * c)
        ops.ew_f32(L.EW_GEGLU_BWD, St["f"], d_f, x2=d_a, cols=4 * c)
        d_n3 = self._t(M, c)
        self._lin_bwd(tb + "ff.net.0.proj.weight", tb + "ff.net.0.proj.bias", d_f, St["n3"], d_n3)
        d_t2 = self._t(M, c)
        self._ln_bwd(St["t2"], tb + "norm3.", lstat[2], d_n3, d_t2, resid=d_t3)
        # attn2 (cross): to_out, attention to the concept tokens, to_q, norm2
        d_o2 = self._t(M, c)
        self._lin_bwd(tb + "attn2.to_out.0.weight", tb + "attn2.to_out.0.bias", d_t2, St["o2"], d_o2)
        d_q2 = self._t(M, c)
        KV, dKV, o = self.KV, self.dKV, s.kv_off
        ops.attention_bwd_f32(St["q2"], KV[:, o:o + c], KV[:, o + c:o + 2 * c], St["o2"], lse[1], d_o2, d_q2,
                              dKV[:, o:o + c], dKV[:, o + c:o + 2 * c], B, s.heads, ntok, self.ex.lu, s.dh)
        d_n2 = self._t(M, c)
        self._lin_bwd(tb + "attn2.to_q.weight", None, d_q2, St["n2"], d_n2)
        d_t1 = self._t(M, c)
        self._ln_bwd(St["t1"], tb + "norm2.", lstat[1], d_n2, d_t1, resid=d_t2)
        # attn1 (self): to_out, attention, q / k / v, norm1
        d_o1 = self._t(M, c)
        self._lin_bwd(tb + "attn1.to_out.0.weight", tb + "attn1.to_out.0.bias", d_t1, St["o1"], d_o1)
        qkv = St["qkv"]
        d_qkv = self._t(M, 3 * c)
        ops.attention_bwd_f32(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], St["o1"], lse[0], d_o1, d_qkv[:, :c],
                              d_qkv[:, c:2 * c], d_qkv[:, 2 * c:], B, s.heads, ntok, ntok, s.dh)
        qkv_names = [tb + "attn1.to_q.weight", tb + "attn1.to_k.weight", tb + "attn1.to_v.weight"]
        d_n1 = self._t(M, c)
        self._lin_bwd(qkv_names[0], None, d_qkv, St["n1"], d_n1, w=self.span(qkv_names).view(3 * c, c),
                      dw=self.Gspan(qkv_names, 3 * c))
        d_t0 = self._t(M, c)
        self._ln_bwd(St["t0"], tb + "norm1.", lstat[0], d_n1, d_t0, resid=d_t1)
        # proj_in, GroupNorm (eps 1e-6, no SiLU); the block's residual x
        d_gn = self._t(M, c)
        self._lin_bwd(p + "proj_in.weight", p + "proj_in.bias", d_t0, St["gn"], d_gn)
        dx = self._t(M, c)
        g = Geom(B, s.h, s.h)
        self._gn_bwd(x, g, p + "norm.", St["stg"], False, d_gn, dx, False, resid=dout)
        return dx
