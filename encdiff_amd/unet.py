"""HIP executor of the EncDiff UNet denoiser (forward + backward), MI355X.

Restates openaimodel_enc.UNetModel.forward (openaimodel_enc.py:712-748) with
ResBlock._forward (:255-275), SpatialTransformer / BasicTransformerBlock /
CrossAttention / GEGLU (attention.py:37-261) as a static schedule of C-ABI kernel
launches over preallocated NHWC bf16 activations.  No torch autograd is used
inside: the backward is written out layer by layer, weight gradients land in the
fp32 arena (split-K slabs summed in a fixed order, one partial-sum reduction for all
norm affine parameters), and only the gradient w.r.t. the context (concept tokens) is
handed back to torch for the as-is concept encoder.

Fusions relative to the reference op graph:
  * GroupNorm + FiLM (1 + scale, shift) + SiLU in one kernel (fwd and bwd),
  * AvgPool2d / nearest x2 of up/down ResBlocks inside the conv's im2col gather,
  * bias, residual adds and the skip path inside GEMM epilogues,
  * all 28 emb_layers projections as ONE GEMM, all 16 cross-attention K/V
    projections of the 20 concept tokens as ONE GEMM (fwd, dgrad and wgrad),
  * q/k/v of self-attention as one [3C] GEMM, heads read in place ('b n (h d)'),
  * each layer's weight- and input-gradient GEMMs as ONE launch (encdiff_gemm_pair).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from . import _lib as L
from . import ops
from .arena import NormPartials, PackTable, ParamArena
from .ops import Geom

BF16 = torch.bfloat16
F32 = torch.float32
GN_EPS = 1e-5      # GroupNorm32 (util.py:227-233)
ST_GN_EPS = 1e-6   # Normalize (attention.py:76-77)
# GroupNorm forward statistics from the producing GEMM's epilogue at >= 8x8 (0: reduce in the
# GroupNorm kernel, for A/B runs)
GN_FROM_PRODUCER = os.environ.get("ENCDIFF_GN_FROM_PRODUCER", "1") != "0"
# a split-K ResBlock conv's finalize folded into the GroupNorm that reads its output: forward
# conv1 -> GN2 in the block, conv2 -> the next block's GN1; backward the conv input gradients
# -> GN2 / GN1 backward, transformer linears -> the LayerNorm / GroupNorm backward reading their
# input gradient.  One launch instead of two (0: separate finalize launches, A/B runs)
GN_FIN = os.environ.get("ENCDIFF_GN_FIN", "1") != "0"
# resampling ResBlocks (cin == cout): the adjoints of conv1's input resample and of the skip branch's
# resample read by the GN1 backward (EncdiffGroupNormArgs.dy_resample / resid_resample) instead of two
# elementwise launches (0: separate launches, A/B)
RS_FUSED = os.environ.get("ENCDIFF_RS_FUSED", "1") != "0"
# grouped weight gradients (ops.WgradGroup): one grid per WG_WINDOW UNet blocks of the backward
# (0: one grid per DP bucket region)
WG_WINDOW = int(os.environ.get("ENCDIFF_WG_WINDOW", "1"))
LN_EPS = 1e-5      # nn.LayerNorm default (attention.py:206-208)
# the row-local SpatialTransformer tail (attn1.to_out .. proj_out) as one kernel
# (encdiff_st_tail_fwd) in no-grad forwards (0: the separate launches, for A/B runs)
ST_TAIL_FUSED = os.environ.get("ENCDIFF_ST_TAIL", "1") != "0"
# inference at sampling batches: ResBlock GroupNorms folded into the convs' A staging
# (_res_fwd_agn); larger batches keep the producer-statistics GroupNorm launches
AGN = os.environ.get("ENCDIFF_AGN", "1") != "0"
# LayerNorm applied in the consuming linear's A staging at inference (c > 128 transformer blocks):
# off by default -- DDIM B=8 606 / 611 -> 600 / 600 steps/s with it (profiles/r04_lna_ab.txt): every
# workgroup re-reduces its rows' statistics and rewrites each staged tile, which costs more than
# the LayerNorm launch it saves at these sizes (the same finding as AGN for the ResBlock convs)
LNA_IN = os.environ.get("ENCDIFF_LNA", "0") == "1"
AGN_MAX_B = int(os.environ.get("ENCDIFF_AGN_MAX_B", "32"))
# ResBlock convs too (else only the fused ST heads): off by default -- DDIM B=8 measured 500 steps/s
# with it vs 595 without (the per-workgroup statistics prologue costs more than the launches it saves)
AGN_RES = os.environ.get("ENCDIFF_AGN_RES", "0") != "0"
AGN_FOLD = os.environ.get("ENCDIFF_AGN_FOLD", "1") != "0"  # split-K combined in the kernel (else a finalize pass)
# inference at sampling batches: each ResBlock as two launches (ops.resconv_fwd: GroupNorm in LDS
# over whole staged images + conv + skip) instead of four to six (0: the unfused launches, A/B)
RC = os.environ.get("ENCDIFF_RC", "1") != "0"
RC_MAX_B = int(os.environ.get("ENCDIFF_RC_MAX_B", "32"))
# ... for images of at most this many elements (pixels x channels): every workgroup re-reduces its
# whole images' statistics, which at configs[4]'s 32x32 x 128+ level (1024 workgroups each reading a
# 256 KB image) made DDIM slower than the separate GroupNorm launches (270 -> 227 steps/s)
RC_MAX_IMG = int(os.environ.get("ENCDIFF_RC_MAX_IMG", "65536"))
# widest level that uses it: at c = 256 one workgroup streams 2.6 MB of weights through one CU
# (74 us at B = 8 against ~35 us for the separate launches, tools/st_tail_bench.py)
ST_TAIL_MAXC = int(os.environ.get("ENCDIFF_ST_TAIL_MAXC", "128"))
# ... also in the training forward, writing the activations the backward reads
ST_TAIL_TRAIN = os.environ.get("ENCDIFF_ST_TAIL_TRAIN", "1") != "0"
# inference, wider blocks (ST_TAIL_MAXC < c <= ST_TAIL_HEAD_MAXC) at sampling batches: the fused
# tail up to norm3 (t2, n3 written), the feed-forward and proj_out as GEMM launches -- one workgroup
# per row tile streaming the 1.5 MB feed-forward weights is what makes the whole tail slow there
ST_TAIL_HEAD = os.environ.get("ENCDIFF_ST_TAIL_HEAD", "1") != "0"
ST_TAIL_HEAD_MAXC = int(os.environ.get("ENCDIFF_ST_TAIL_HEAD_MAXC", "256"))
ST_TAIL_HEAD_MAX_B = int(os.environ.get("ENCDIFF_ST_TAIL_HEAD_MAX_B", "32"))
# ... and in the training forward, saving the activations up to norm3 for the (unfused) backward
ST_TAIL_HEAD_TRAIN = os.environ.get("ENCDIFF_ST_TAIL_HEAD_TRAIN", "1") != "0"
# A/B: the c = 128 training tail in head mode too (up to norm3; the GEGLU feed-forward and proj_out
# as GEMM launches, which share the weights across row tiles instead of streaming them per tile)
ST_TAIL_C128_HEAD = os.environ.get("ENCDIFF_ST_TAIL_C128_HEAD", "0") == "1"
# ... and their head (GroupNorm statistics from x, proj_in, norm1, q/k/v) as one kernel too: off by
# default -- DDIM B=8 716 -> 705 steps/s with it (8 workgroups at the 4x4 level each stream the
# 512 KB of proj_in + q/k/v weights; the GroupNorm + GEMM + LayerNorm + GEMM launches spread them)
ST_HEAD_256 = os.environ.get("ENCDIFF_ST_HEAD_256", "0") != "0"
# training backward of the SpatialTransformers at c <= ST_BWD_MAXC as fused kernels: the tail's
# input-gradient chain (encdiff_st_tail_bwd), the self-attention backward, the head's chain
# (encdiff_st_head_bwd), the block's 8 weight gradients as ONE grouped launch, the GroupNorm
# backward -- 5 launches instead of 14 (the weight-gradient fold rides in the GroupNorm backward;
# 0: the per-layer launches, for A/B runs)
ST_BWD = os.environ.get("ENCDIFF_ST_BWD", "1") != "0"
ST_BWD_MAXC = int(os.environ.get("ENCDIFF_ST_BWD_MAXC", "128"))
# the fused blocks' weight gradients: "st" (encdiff_st_wgrad: large output blocks, each operand read
# about once, + a chunk fold), "group" (the generic grouped launch's 64 x 64 parts) or "single"
# (standalone split-K launches), for A/B
ST_BWD_WG = os.environ.get("ENCDIFF_ST_BWD_WG", "st")
# ... and their chunk fold as extra workgroups of the block's GroupNorm backward (the next launch;
# the fold is off its critical path) instead of a launch of its own (0: separate, A/B)
ST_FOLD_RIDE = os.environ.get("ENCDIFF_ST_FOLD_RIDE", "1") != "0"
# training forward: the SiLU GroupNorms also store silu'(z) (bf16), which their backward reads instead
# of recomputing two transcendentals per element in its VALU-bound first pass -- measured slower
# (8.93 -> 8.975 ms/step: the backward stayed at ~8.3 us per call, the forward grew), so off by default
GN_DSILU = os.environ.get("ENCDIFF_GN_DSILU", "0") == "1"


# --------------------------------------------------------------------------- spec
@dataclass
class ResSpec:
    prefix: str
    cin: int
    cout: int
    updown: int          # RESAMPLE_NONE / DOWN2 / UP2
    hin: int
    hout: int
    film_off: int = 0


@dataclass
class STSpec:
    prefix: str
    c: int
    heads: int
    dh: int
    h: int
    kv_off: int = 0
    fp8: bool = False  # self-attention scores on fp8 MFMA (UNetModel attn_fp8_min_tokens)


@dataclass
class ConvSpec:
    prefix: str
    cin: int
    cout: int
    h: int


@dataclass
class UNetSpec:
    cfg: dict
    input_blocks: List[list] = field(default_factory=list)
    middle: list = field(default_factory=list)
    output_blocks: List[list] = field(default_factory=list)
    res: List[ResSpec] = field(default_factory=list)
    sts: List[STSpec] = field(default_factory=list)
    skip_ch: List[int] = field(default_factory=list)
    film_total: int = 0
    kv_total: int = 0

    @staticmethod
    def from_config(cfg: dict) -> "UNetSpec":
        """openaimodel_enc.py:507-688 for the configuration family the path uses:
        use_spatial_transformer=True, use_scale_shift_norm=True, resblock_updown=True,
        legacy=True, transformer_depth=1, num_head_channels=-1."""
        mc, heads = cfg["model_channels"], cfg["num_heads"]
        attn, nrb, mult = list(cfg["attention_resolutions"]), cfg["num_res_blocks"], list(cfg["channel_mult"])
        H = cfg["image_size"]
        s = UNetSpec(cfg=dict(cfg))
        s.input_blocks.append([ConvSpec("input_blocks.0.0.", cfg["in_channels"], mc, H)])
        chans = [mc]
        ch, ds, h = mc, 1, H

        def res(prefix, cin, cout, ud, hin):
            hout = hin // 2 if ud == L.RESAMPLE_DOWN2 else (hin * 2 if ud == L.RESAMPLE_UP2 else hin)
            r = ResSpec(prefix, cin, cout, ud, hin, hout, film_off=s.film_total)
            s.film_total += 2 * cout
            s.res.append(r)
            return r

        fp8_min = cfg.get("attn_fp8_min_tokens") or 0

        def st(prefix, c, hh):
            t = STSpec(prefix, c, heads, c // heads, hh, kv_off=s.kv_total,
                       fp8=bool(fp8_min) and hh * hh >= fp8_min)
            s.kv_total += 2 * c
            s.sts.append(t)
            return t

        for level, m in enumerate(mult):
            for _ in range(nrb):
                i = len(s.input_blocks)
                blk = [res(f"input_blocks.{i}.0.", ch, m * mc, 0, h)]
                ch = m * mc
                if ds in attn:
                    blk.append(st(f"input_blocks.{i}.1.", ch, h))
                s.input_blocks.append(blk)
                chans.append(ch)
            if level != len(mult) - 1:
                i = len(s.input_blocks)
                s.input_blocks.append([res(f"input_blocks.{i}.0.", ch, ch, L.RESAMPLE_DOWN2, h)])
                h //= 2
                chans.append(ch)
                ds *= 2
        s.middle = [res("middle_block.0.", ch, ch, 0, h), st("middle_block.1.", ch, h),
                    res("middle_block.2.", ch, ch, 0, h)]
        s.skip_ch = list(chans)
        for level, m in list(enumerate(mult))[::-1]:
            for i in range(nrb + 1):
                j = len(s.output_blocks)
                ich = chans.pop()
                blk = [res(f"output_blocks.{j}.0.", ch + ich, mc * m, 0, h)]
                ch = mc * m
                if ds in attn:
                    blk.append(st(f"output_blocks.{j}.{len(blk)}.", ch, h))
                if level and i == nrb:
                    blk.append(res(f"output_blocks.{j}.{len(blk)}.", ch, ch, L.RESAMPLE_UP2, h))
                    h *= 2
                    ds //= 2
                s.output_blocks.append(blk)
        s.out_ch = ch
        return s

    # ---------------------------------------------------------------- arena order
    def conv_weights(self):
        """3x3 conv weights run by the GEMM engine (stored channels-last in the arena)."""
        out = []
        for r in self.res:
            out += [r.prefix + "in_layers.2.weight", r.prefix + "out_layers.3.weight"]
        return out

    def arena_order(self, named: Dict[str, torch.nn.Parameter]):
        """Arena layout: [emb W][emb b][cross K/V W][per-ST qkv W]...rest (named order)."""
        order = []
        taken = set()

        def take(n):
            order.append((n, named[n]))
            taken.add(n)
        for r in self.res:
            take(r.prefix + "emb_layers.1.weight")
        for r in self.res:
            take(r.prefix + "emb_layers.1.bias")
        for t in self.sts:
            tb = t.prefix + "transformer_blocks.0.attn2."
            take(tb + "to_k.weight")
            take(tb + "to_v.weight")
        for t in self.sts:
            tb = t.prefix + "transformer_blocks.0.attn1."
            for w in ("to_q", "to_k", "to_v"):
                take(tb + w + ".weight")
        for n, p in named.items():
            if n not in taken:
                order.append((n, p))
        return order


# --------------------------------------------------------------------------- executor
class UNetExecutor:
    """Binds a UNetSpec to a ParamArena; owns the bf16 packed weights, the norm
    partial-sum matrix and (per batch size) the activation buffers."""

    def __init__(self, spec: UNetSpec, arena: ParamArena):
        self.spec = spec
        self.arena = arena
        self.dev = arena.device
        cfg = spec.cfg
        self.mc = cfg["model_channels"]
        self.cd = cfg["context_dim"]
        self.lu = cfg["latent_unit"]
        self.H = cfg["image_size"]
        a = arena
        pk = PackTable(arena)
        # fused groups
        emb_w = [r.prefix + "emb_layers.1.weight" for r in spec.res]
        o, n = a.span(emb_w)
        pk.add("emb_all", o, spec.film_total, 4 * self.mc)
        self.emb_bias_names = [r.prefix + "emb_layers.1.bias" for r in spec.res]
        ob, nb = a.span(self.emb_bias_names)
        self.emb_bias = a.master[ob:ob + nb]
        self.emb_bias_grad = a.grad[ob:ob + nb]
        self.emb_w_grad = a.grad[o:o + n].view(spec.film_total, 4 * self.mc)
        kv_w = []
        for t in spec.sts:
            tb = t.prefix + "transformer_blocks.0.attn2."
            kv_w += [tb + "to_k.weight", tb + "to_v.weight"]
        o, n = a.span(kv_w)
        pk.add("kv_all", o, spec.kv_total, self.cd)
        self.kv_w_grad = a.grad[o:o + n].view(spec.kv_total, self.cd)
        self.qkv_grad = {}
        for t in spec.sts:
            tb = t.prefix + "transformer_blocks.0.attn1."
            o, n = a.span([tb + "to_q.weight", tb + "to_k.weight", tb + "to_v.weight"])
            pk.add(t.prefix + "qkv", o, 3 * t.c, t.c)
            self.qkv_grad[t.prefix] = a.grad[o:o + n].view(3 * t.c, t.c)
        # plain GEMM weights
        pk.add("time_embed.0.weight", a.offsets["time_embed.0.weight"][0], 4 * self.mc, self.mc)
        # input conv (3 -> mc): [mc][3][3][3] -> [mc][9 taps][8] (channel-padded GEMM B layout)
        cin0 = spec.input_blocks[0][0].cin
        assert cin0 <= 8
        pk.add("input_conv", a.offsets["input_blocks.0.0.weight"][0], self.mc, 72, kind=2, cin=cin0)
        pk.add("time_embed.2.weight", a.offsets["time_embed.2.weight"][0], 4 * self.mc, 4 * self.mc)
        for r in spec.res:
            for w, cin in (("in_layers.2.weight", r.cin), ("out_layers.3.weight", r.cout)):
                # arena stores these [co][kh][kw][ci] (channels_last) -> identity pack
                kind = 0 if (r.prefix + w) in a.cl else 1
                pk.add(r.prefix + w, a.offsets[r.prefix + w][0], r.cout, 9 * cin, kind=kind, cin=cin)
            if r.cin != r.cout:
                pk.add(r.prefix + "skip_connection.weight", a.offsets[r.prefix + "skip_connection.weight"][0],
                       r.cout, r.cin)
        for t in spec.sts:
            c = t.c
            tb = t.prefix + "transformer_blocks.0."
            for w, rows, cols in (("proj_in.weight", c, c), ("proj_out.weight", c, c)):
                pk.add(t.prefix + w, a.offsets[t.prefix + w][0], rows, cols)
            for w, rows, cols in (("attn1.to_out.0.weight", c, c), ("attn2.to_q.weight", c, c),
                                  ("attn2.to_out.0.weight", c, c), ("ff.net.0.proj.weight", 8 * c, c),
                                  ("ff.net.2.weight", c, 4 * c)):
                pk.add(tb + w, a.offsets[tb + w][0], rows, cols)
        # the fused transformer backward reads every Linear of its block transposed ([in][out]):
        # packed by the same per-step pack launch (kind 6)
        # (the kernels' support: c in {64, 128}, 8 heads, <= 64 concept tokens, whole row tiles per image)
        self.stf = {t.prefix for t in spec.sts
                    if ST_BWD and t.c <= ST_BWD_MAXC and t.heads == 8 and self.lu <= 64 and
                    ((t.c == 64 and t.h * t.h % 64 == 0) or (t.c == 128 and t.h * t.h % 32 == 0))}
        for t in spec.sts:
            if t.prefix not in self.stf:
                continue
            c, tb = t.c, t.prefix + "transformer_blocks.0."
            for key, name, rows, cols in (("po", t.prefix + "proj_out.weight", c, c), ("in", t.prefix + "proj_in.weight", c, c),
                                          ("ff2", tb + "ff.net.2.weight", c, 4 * c),
                                          ("ff1", tb + "ff.net.0.proj.weight", 8 * c, c),
                                          ("out2", tb + "attn2.to_out.0.weight", c, c), ("q2", tb + "attn2.to_q.weight", c, c),
                                          ("out1", tb + "attn1.to_out.0.weight", c, c)):
                pk.add(t.prefix + "T:" + key, a.offsets[name][0], rows, cols, kind=6)
            o, _ = a.span([tb + "attn1.to_q.weight", tb + "attn1.to_k.weight", tb + "attn1.to_v.weight"])
            pk.add(t.prefix + "T:qkv", o, 3 * c, c, kind=6)
        pk.finalize()
        self.pack = pk
        # norm partials: GN rows = batch (set at bind time), LN rows = LN_PARTS
        self._gn_names = []
        for r in spec.res:
            self._gn_names.append((r.prefix + "in_layers.0.weight", r.prefix + "in_layers.0.bias"))
            self._gn_names.append((r.prefix + "out_layers.0.weight", r.prefix + "out_layers.0.bias"))
        for t in spec.sts:
            self._gn_names.append((t.prefix + "norm.weight", t.prefix + "norm.bias"))
        self._gn_names.append(("out.0.weight", "out.0.bias"))
        # output-block / out columns last: the split backward folds that suffix early
        self._gn_names.sort(key=lambda p: self._early_final(p[0]))
        # LayerNorm partials: the per-layer backward kernels' (LN_PARTS rows); the fused transformer
        # backward's (one row per row tile, per batch size: self.ln_f, bind)
        self.ln = NormPartials(arena, ops.LN_PARTS)
        for t in spec.sts:
            if t.prefix in self.stf:
                continue
            tb = t.prefix + "transformer_blocks.0."
            for nn_ in ("norm1", "norm2", "norm3"):
                self.ln.add(tb + nn_ + ".weight", tb + nn_ + ".bias")
        self.ln.finalize()
        self._stwg = ops.WgradGroup()  # the fused transformer blocks' weight gradients (ST_BWD_WG "group")
        self._stwgk = ops.StWgrad()    # ... (ST_BWD_WG "st": encdiff_st_wgrad)
        self.gn: Optional[NormPartials] = None
        self.B = None
        self._sets: Dict[int, dict] = {}
        self.split_requested = False  # data-parallel trainer: backward(split=True) via autograd
        self.want_dx = False  # backward also writes d x_t (self.d_x): set by _UNetFn when x requires grad
        self.infer = False  # no backward follows the next forward (UNetModel.forward under no_grad)
        # sampling loops (ddim.DDIMSampler's whole-loop graph): samp_ts = the loop's timesteps
        # (S,), samp_i = the step being run.  Step 0 fills the loop's FiLM table (the time MLP and
        # emb_layers for all S timesteps in one pass, one row per step -- every row of a sampling
        # batch has the same t) and the concept tokens' K / V; later steps skip both
        self.samp_ts: Optional[torch.Tensor] = None
        self.samp_i: Optional[int] = None
        self._samp_tabs: Dict[tuple, dict] = {}  # (S, B) -> buffers; graphs hold their addresses
        self._wgg = ops.WgradGroup()  # the backward's grouped weight gradients (planned per batch size)
        self.stat_slots = ops.StatSlots()  # producer-statistics slots the transformer tails add into
        # names shared by every batch size; everything bind() (re)creates is per batch size and is
        # kept in / restored from self._sets -- the GroupNorm partials (rows = B) included: excluded
        # from the shared names although declared above, else a switch back to a larger batch kept
        # the smaller batch's partial rows and its GroupNorm backwards wrote past them.  bind()
        # checks that it rebinds no shared name (_check_shared), so a future per-batch buffer
        # declared in __init__ fails at its first bind instead of writing past a smaller batch's
        self._base_names = (set(self.__dict__) - self._PER_BATCH) | {"_base_names"}
        self.pack.repack()

    _PER_BATCH = frozenset({"gn"})  # declared in __init__, rebound per batch size by bind()
    _SHARED_REBIND = frozenset({"B"})  # shared names bind() itself may reassign

    def _shared_snapshot(self) -> dict:
        return {n: self.__dict__[n] for n in self._base_names if n in self.__dict__}

    def _check_shared(self, before: dict):
        """Per-batch state safe by construction: every name bind() (re)assigns must be per batch
        size (saved / restored across batch switches).  A shared name -- one present after
        __init__ and not in _PER_BATCH -- that bind() rebinds would be kept from the batch size
        bound last, e.g. a B-row buffer reused at a larger B."""
        bad = sorted(n for n, v in before.items()
                     if n not in self._SHARED_REBIND and self.__dict__.get(n) is not v)
        if bad:
            raise RuntimeError(f"UNetExecutor.bind rebinds shared attribute(s) {bad}: per-batch state declared in "
                               "__init__ must be listed in UNetExecutor._PER_BATCH")

    # ---------------------------------------------------------------- helpers
    def W(self, key):
        return self.pack.view(key)

    def P(self, name):
        return self.arena.f32(name)

    def G(self, name):
        return self.arena.grad_of(name)

    def conv_wgrad(self, dy, x, g, cin, name, db, resample=0):
        if name in self.arena.cl:
            ops.conv3x3_wgrad_cl(dy, x, g, cin, self.arena.raw(self.arena.grad, name), db, resample=resample)
        else:
            ops.conv3x3_wgrad(dy, x, g, cin, self.G(name), db, resample=resample)

    def _t(self, rows, cols, dtype=BF16):  # noqa: D401
        return torch.empty(rows, cols, device=self.dev, dtype=dtype)

    # ---------------------------------------------------------------- buffers
    def bind(self, B: int):
        """Allocate every activation / gradient buffer for batch size B (static shapes)."""
        if self.B == B:
            return
        if self.B is not None:  # keep one buffer set per batch size (training B, sampling B ...)
            self._sets[self.B] = {n: v for n, v in self.__dict__.items() if n not in self._base_names}
        self.B = B
        if B in self._sets:
            self.__dict__.update(self._sets[B])
            return
        shared = self._shared_snapshot()
        self._bind_new(B)
        self._check_shared(shared)

    def _bind_new(self, B: int):
        ops.ensure_scratch(self.dev.index if self.dev.index is not None else None)
        sp = self.spec
        self._split = False  # split_plan() not computed for this batch size yet
        self._cont = None
        self.gn = NormPartials(self.arena, B)
        for gname, bname in self._gn_names:
            self.gn.add(gname, bname)
        self.gn.finalize()
        # the fused transformer backward's LayerNorm partials: a row per row tile (tiles >= 32 rows)
        self.ln_f = NormPartials(self.arena, max([B * st.h * st.h // 32 for st in sp.sts if st.prefix in self.stf] or [1]))
        for st in sp.sts:
            if st.prefix in self.stf:
                tb = st.prefix + "transformer_blocks.0."
                for nn_ in ("norm1", "norm2", "norm3"):
                    self.ln_f.add(tb + nn_ + ".weight", tb + nn_ + ".bias")
        self.ln_f.finalize()
        t = self._t
        mc, H = self.mc, self.H
        self.temb0 = t(B, mc); self.th1 = t(B, 4 * mc); self.ta1 = t(B, 4 * mc)
        self.emb = t(B, 4 * mc); self.emb_s = t(B, 4 * mc)
        self.E = t(B, sp.film_total, F32)
        self.dE = t(B, sp.film_total, F32)
        self.dE16 = t(B, sp.film_total)
        self.d_emb_s = t(B, 4 * mc); self.d_emb = t(B, 4 * mc); self.d_ta1 = t(B, 4 * mc); self.d_th1 = t(B, 4 * mc)
        self.ctx16 = t(B * self.lu, self.cd)
        self.KV = t(B * self.lu, sp.kv_total)
        self.dKV = t(B * self.lu, sp.kv_total)
        # per-layer state
        self.state: Dict[str, dict] = {}
        for blk in sp.input_blocks + [sp.middle] + sp.output_blocks:
            for layer in blk:
                if isinstance(layer, ResSpec):
                    self.state[layer.prefix] = self._res_bufs(layer, B)
                elif isinstance(layer, STSpec):
                    self.state[layer.prefix] = self._st_bufs(layer, B)
        g0 = Geom(B, H, H)
        self.h0 = t(g0.pixels, mc)
        # output-block concat inputs and their grads
        self.xcat, self.dxcat = [], []
        for blk in sp.output_blocks:
            r0 = blk[0]
            n = B * r0.hin * r0.hin
            self.xcat.append(t(n, r0.cin))
            self.dxcat.append(t(n, r0.cin))
        # skip connections and the decoder path are written straight into the concat inputs:
        # the last layer of input block i writes the upper channel slice of the output block
        # that consumes it, the layer before each output block its lower slice
        # (torch.cat([h, hs.pop()], 1), openaimodel_enc.py:740, without the copies)
        nhs = len(sp.input_blocks)
        for i in range(nhs):
            j = nhs - 1 - i
            c1 = sp.output_blocks[j][0].cin - sp.skip_ch[i]
            view = self.xcat[j][:, c1:]
            if i == 0:
                self.h0 = view
            else:
                self.state[sp.input_blocks[i][-1].prefix]["out"] = view
        prev_last = sp.middle[-1]
        for j, blk in enumerate(sp.output_blocks):
            c1 = blk[0].cin - sp.skip_ch[nhs - 1 - j]
            self.state[prev_last.prefix]["out"] = self.xcat[j][:, :c1]
            prev_last = blk[-1]
        self.x8 = t(g0.pixels, 8)           # x_t as channel-padded bf16 rows (input conv operand)
        self.dw_in = t(self.mc, 72, F32)     # input conv weight gradient, GEMM layout
        self.deps8 = t(g0.pixels, 8)         # d eps as channel-padded bf16 rows
        self.dw_out = t(8, 9 * sp.out_ch, F32)
        self.db_out = torch.zeros(8, device=self.dev, dtype=F32)  # bias-gradient accumulator (left zero)
        self.a_out = t(g0.pixels, sp.out_ch)
        self.ds_out = t(g0.pixels, sp.out_ch) if GN_DSILU else None
        self.st_out = t(B, 64, F32)
        self.d_aout = t(g0.pixels, sp.out_ch)
        self.d_hlast = t(g0.pixels, sp.out_ch)
        self.eps = torch.empty(B, self.spec.cfg["out_channels"], H, H, device=self.dev, dtype=F32)
        self.d_ctx = torch.empty(B, self.lu * self.cd, device=self.dev, dtype=F32)
        # per-level scratch for transformer backward
        self.st_scratch = {}
        for t_ in sp.sts:
            key = (t_.h, t_.c)
            if key in self.st_scratch:
                continue
            M = B * t_.h * t_.h
            c = t_.c
            self.st_scratch[key] = dict(d_a=t(M, 4 * c), d_n=t(M, c), d_o=t(M, c), d_g=t(M, c))
            if t_.prefix in self.stf:  # the fused backward's cross-attention dK / dV partial slabs
                self.st_scratch[key]["kv_part"] = t(M // 32 * self.lu, 2 * c, F32)
        self.res_scratch = {}
        self._bind_gn_stats(B)

    def _bind_gn_stats(self, B):
        """GroupNorm statistics from the producers: every tensor a GroupNorm forward reads at
        >= 8x8 (layer outputs, the concat inputs, each ResBlock's conv1 output) gets a
        [2 * pixels/64][C] fp32 buffer that its producing GEMM fills with per-64-row-segment
        channel sums (EncdiffGemmArgs.gn_stats); a concat input's two producers fill their
        channel ranges of one buffer.  Keyed by the tensor's data pointer."""
        self.gst = {}
        if not GN_FROM_PRODUCER or B < 64:  # small (sampling) batches: the producers keep split-K
            return
        sp = self.spec

        def add(x, hw, key_views=()):
            if hw < 64:
                return
            st = self._t(2 * x.shape[0] // 64, x.shape[1], F32)
            self.gst[x.data_ptr()] = st
            for v in key_views:
                off = v.data_ptr() - x.data_ptr()
                self.gst[v.data_ptr()] = st[:, off // x.element_size():]
        nhs = len(sp.input_blocks)
        for j, blk in enumerate(sp.output_blocks):
            c1 = blk[0].cin - sp.skip_ch[nhs - 1 - j]
            add(self.xcat[j], blk[0].hin ** 2, (self.xcat[j][:, c1:],))
        for blk in sp.input_blocks + [sp.middle] + sp.output_blocks:
            for layer in blk:
                if not isinstance(layer, (ResSpec, STSpec)):
                    continue  # the input conv (its output h0 is a concat view)
                S = self.state[layer.prefix]
                hw = (layer.hout if isinstance(layer, ResSpec) else layer.h) ** 2
                if S["out"].data_ptr() not in self.gst:
                    add(S["out"], hw)
                if isinstance(layer, ResSpec):
                    add(S["h1"], layer.hout ** 2)

    def _gst(self, x):
        """The producer-statistics buffer of tensor x (None: the GroupNorm reduces itself)."""
        return self.gst.get(x.data_ptr())

    def _res_bufs(self, r: ResSpec, B):
        t = self._t
        Mi, Mo = B * r.hin * r.hin, B * r.hout * r.hout
        d = dict(a1=t(Mi, r.cin), st1=t(B, 64, F32), h1=t(Mo, r.cout), a2=t(Mo, r.cout), st2=t(B, 64, F32),
                 out=t(Mo, r.cout), d_a2=t(Mo, r.cout), d_h1=t(Mo, r.cout), d_in=t(Mi, r.cin), d_a1=t(Mi, r.cin))
        if GN_DSILU:  # silu'(z) of GN1 / GN2 (training forward -> backward)
            d["ds1"], d["ds2"] = t(Mi, r.cin), t(Mo, r.cout)
        if r.updown:
            d["d_a1r"] = t(Mo, r.cin)
        if r.updown == L.RESAMPLE_DOWN2:
            d["a1r"] = t(Mo, r.cin)  # AvgPool2d(2) of the GN1 output (the conv's input)
        if r.updown and r.cin == r.cout:
            d["xr"] = t(Mo, r.cout)
        return d

    def _st_bufs(self, s: STSpec, B):
        t = self._t
        M = B * s.h * s.h
        c = s.c
        # gradients the weight-gradient GEMMs read get a buffer of their own (written once per
        # step; LayerNorm backward adds its residual branch out of place)
        return dict(gn=t(M, c), stg=t(B, 64, F32), t0=t(M, c), n1=t(M, c), s1=t(M, 2, F32), qkv=t(M, 3 * c),
                    o1=t(M, c), lse1=t(B * s.heads, s.h * s.h, F32), t1=t(M, c), n2=t(M, c), s2=t(M, 2, F32),
                    q2=t(M, c), o2=t(M, c), lse2=t(B * s.heads, s.h * s.h, F32), t2=t(M, c), n3=t(M, c),
                    s3=t(M, 2, F32), f=t(M, 8 * c), a=t(M, 4 * c), t3=t(M, c), out=t(M, c), d_in=t(M, c),
                    d_t3=t(M, c), d_t2=t(M, c), d_t1=t(M, c), d_t0=t(M, c), d_f=t(M, 8 * c), d_q2=t(M, c),
                    d_qkv=t(M, 3 * c))

    # ---------------------------------------------------------------- forward
    def _samp_table(self, B: int) -> dict:
        """The sampling loop's per-step FiLM rows (S, film_total) fp32 and the time-MLP buffers
        of its S timesteps, per (S, B); kept for the life of the executor."""
        S = int(self.samp_ts.shape[0])
        tab = self._samp_tabs.get((S, B))
        if tab is None:
            mc, dev = self.mc, self.samp_ts.device
            bf = dict(device=dev, dtype=torch.bfloat16)
            tab = dict(temb0=torch.empty(S, mc, **bf), th1=torch.empty(S, 4 * mc, **bf),
                       ta1=torch.empty(S, 4 * mc, **bf), emb=torch.empty(S, 4 * mc, **bf),
                       emb_s=torch.empty(S, 4 * mc, **bf),
                       E=torch.empty(S, self.spec.film_total, device=dev, dtype=torch.float32))
            self._samp_tabs[(S, B)] = tab
        return tab

    def _samp_fill(self, tab: dict, B: int):
        """Time MLP + emb_layers over the loop's S timesteps at once.  Each GEMM takes the plan
        of the B-row problem a step would run (plan_m=B), so every row is bitwise the FiLM row the
        step's own forward computes."""
        mc = self.mc
        ops.timestep_embedding(self.samp_ts, mc, tab["temb0"])
        ops.linear_fwd(tab["temb0"], self.W("time_embed.0.weight"), tab["th1"], bias=self.P("time_embed.0.bias"),
                       plan_m=B)
        ops.ew(L.EW_SILU, tab["th1"], tab["ta1"])
        ops.linear_fwd(tab["ta1"], self.W("time_embed.2.weight"), tab["emb"], bias=self.P("time_embed.2.bias"),
                       plan_m=B)
        ops.ew(L.EW_SILU, tab["emb"], tab["emb_s"])
        ops.linear_fwd(tab["emb_s"], self.W("emb_all"), tab["E"], bias=self.emb_bias, out_f32=True, plan_m=B)

    def forward(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        """x (B,C,H,W) fp32, t (B,) int64, ctx (B, latent_unit*context_dim) fp32 -> eps (B,C,H,W) fp32."""
        B = x.shape[0]
        self.bind(B)
        sp, mc = self.spec, self.mc
        self._pend = None  # GemmArgs of a ResBlock output whose split-K finalize is deferred
        self._x = x.contiguous()
        self._t_in = t.contiguous()
        samp = self.samp_ts is not None and self.samp_i is not None and self.infer
        if samp:
            tab = self._samp_table(B)
            if self.samp_i == 0:
                self._samp_fill(tab, B)
            row = tab["E"][self.samp_i]
            self._E_use, self._E_ld = row.unsqueeze(0).expand(B, row.shape[0]), 0
        else:
            # timestep embedding + time MLP (openaimodel_enc.py:726-727)
            ops.timestep_embedding(self._t_in, mc, self.temb0)
            ops.linear_fwd(self.temb0, self.W("time_embed.0.weight"), self.th1, bias=self.P("time_embed.0.bias"))
            ops.ew(L.EW_SILU, self.th1, self.ta1)
            ops.linear_fwd(self.ta1, self.W("time_embed.2.weight"), self.emb, bias=self.P("time_embed.2.bias"))
            ops.ew(L.EW_SILU, self.emb, self.emb_s)
            # all 28 emb_layers at once (fp32 FiLM table)
            ops.linear_fwd(self.emb_s, self.W("emb_all"), self.E, bias=self.emb_bias, out_f32=True)
            self._E_use, self._E_ld = self.E, self.E.shape[1]
        if not samp or self.samp_i == 0:
            # concept tokens -> every cross-attention's K/V at once
            ctx2 = ctx.contiguous().view(B * self.lu, self.cd)
            ops.ew(L.EW_F32_TO_BF16, ctx2, self.ctx16)
            ops.linear_fwd(self.ctx16, self.W("kv_all"), self.KV)
        # input conv
        g0 = Geom(B, self.H, self.H)
        # input conv on the GEMM engine over channel-padded rows (openaimodel_enc.py:494)
        ops.nchw_to_rows(self._x, 8, self.x8)
        ops.conv3x3_fwd(self.x8, g0, 8, self.W("input_conv"), self.h0, bias=self.P("input_blocks.0.0.bias"),
                        gn_stats=self._gst(self.h0))
        hs = [self.h0]
        h = self.h0
        for blk in sp.input_blocks[1:]:
            for layer in blk:
                h = self._layer_fwd(layer, h)
            hs.append(h)
        for layer in sp.middle:
            h = self._layer_fwd(layer, h)
        self._hs = hs
        for j, blk in enumerate(sp.output_blocks):
            skip = hs[len(hs) - 1 - j]
            xc = self.xcat[j]
            c1 = h.shape[1]
            # both halves were written in place by their producers (see bind)
            assert h.data_ptr() == xc.data_ptr() and skip.data_ptr() == xc[:, c1:].data_ptr()
            h = xc
            for layer in blk:
                h = self._layer_fwd(layer, h)
        self._h_last = h
        ops.groupnorm_fwd(h, g0, self.P("out.0.weight"), self.P("out.0.bias"), self.a_out, self.st_out, GN_EPS, True,
                          in_stats=self._gst(h), x_from=self._take_pend(h), dsilu=None if self.infer else self.ds_out)
        ops.small_conv_out_fwd(self.a_out, g0, self.P("out.2.weight"), self.P("out.2.bias"), self.eps)
        return self.eps

    def _take_pend(self, x):
        """The deferred finalize of x's producer when the GroupNorm about to read x can combine
        its slabs (x is exactly that GEMM's output); any other pending finalize runs now."""
        p, self._pend = self._pend, None
        if p is None:
            return None
        if p.c == x.data_ptr() and p.N == x.shape[1] and p.ldc == x.stride(0) and self._gst(x) is None:
            return p
        ops.finalize(p)
        return None

    def _layer_fwd(self, layer, x):
        if isinstance(layer, ResSpec):
            return self._res_fwd(layer, x)
        return self._st_fwd(layer, x)  # (it takes or finalizes a pending finalize of x)

    def _res_fwd(self, r: ResSpec, x):
        """openaimodel_enc.py:255-275 with use_scale_shift_norm."""
        B = self.B
        S = self.state[r.prefix]
        S["x"] = x
        gi, go = Geom(B, r.hin, r.hin), Geom(B, r.hout, r.hout)
        if self.infer and RC and B <= RC_MAX_B and self._res_fwd_rc(r, S, x, gi, go):
            return S["out"]
        if self.infer and AGN and AGN_RES and B <= AGN_MAX_B:
            return self._res_fwd_agn(r, S, x, gi, go)
        ops.groupnorm_fwd(x, gi, self.P(r.prefix + "in_layers.0.weight"), self.P(r.prefix + "in_layers.0.bias"),
                          S["a1"], S["st1"], GN_EPS, True, in_stats=self._gst(x), x_from=self._take_pend(x),
                          dsilu=None if self.infer else S.get("ds1"))
        a1, rs = self._conv1_input(r, S, go)
        f1 = ops.conv3x3_fwd(a1, go, r.cin, self.W(r.prefix + "in_layers.2.weight"), S["h1"],
                             bias=self.P(r.prefix + "in_layers.2.bias"), resample=rs, gn_stats=self._gst(S["h1"]),
                             defer=GN_FIN and self._gst(S["h1"]) is None)
        film = self._E_use[:, r.film_off:]
        ops.groupnorm_fwd(S["h1"], go, self.P(r.prefix + "out_layers.0.weight"), self.P(r.prefix + "out_layers.0.bias"),
                          S["a2"], S["st2"], GN_EPS, True, film=film, ld_film=self._E_ld,
                          in_stats=self._gst(S["h1"]), x_from=f1, dsilu=None if self.infer else S.get("ds2"))
        # skip path into the output buffer, then conv2 adds onto it
        out = S["out"]
        if r.cin != r.cout:
            ops.linear_fwd(x, self.W(r.prefix + "skip_connection.weight"), out,
                           bias=self.P(r.prefix + "skip_connection.bias"))
            resid = out
        elif r.updown:
            ops.resample(x, S["xr"], go, r.updown)
            resid = S["xr"]
        else:
            resid = x
        # (deferred: the next ResBlock's GN1 or the output GroupNorm combines the slabs, any
        # other reader finalizes first -- _take_pend / _layer_fwd)
        self._pend = ops.conv3x3_fwd(S["a2"], go, r.cout, self.W(r.prefix + "out_layers.3.weight"), out,
                                     bias=self.P(r.prefix + "out_layers.3.bias"), resid=resid, gn_stats=self._gst(out),
                                     defer=GN_FIN and self._gst(out) is None)
        return out

    def _res_fwd_rc(self, r: ResSpec, S, x, gi: Geom, go: Geom) -> bool:
        """Inference ResBlock as two ops.resconv_fwd launches: h1 = conv1(resample(SiLU(GN1(x)))) + b1,
        out = conv2(SiLU(GN2(h1)(1 + scale) + shift)) + b2 + skip(x) -- each conv stages the whole
        images it reads in LDS and normalises them there, so no GroupNorm launch, no normalised
        activation in memory and no skip / resample launch.  x complete first (a producer that
        deferred its finalize finalizes now).  False (nothing launched) outside the kernel's
        support: the caller runs the unfused launches."""
        pre = r.prefix
        w1, w2 = self.W(pre + "in_layers.2.weight"), self.W(pre + "out_layers.3.weight")
        film = self._E_use[:, r.film_off:]
        cskip = r.cin if r.cin != r.cout else 0
        if r.hin * r.hin * r.cin > RC_MAX_IMG or r.hout * r.hout * r.cout > RC_MAX_IMG:
            return False
        # the kernel reads its skip input at the OUTPUT resolution: a channel-changing skip of a
        # resampling block (none in the reference's UNets) stays on the unfused launches
        if cskip and r.updown:
            return False
        # it writes no producer statistics: a later GroupNorm reading S['h1'] / S['out'] from
        # them (GN_FROM_PRODUCER at B >= 64) needs the unfused launches
        if self._gst(S["h1"]) is not None or self._gst(S["out"]) is not None:
            return False
        if cskip:
            skip = dict(xskip=x, wskip=self.W(pre + "skip_connection.weight"), bskip=self.P(pre + "skip_connection.bias"))
        else:
            skip = dict(resid=x, resid_resample=r.updown)
        conv1 = dict(x=x, g=gi, w=w1, y=S["h1"], gamma=self.P(pre + "in_layers.0.weight"),
                     beta=self.P(pre + "in_layers.0.bias"), eps=GN_EPS, bias=self.P(pre + "in_layers.2.bias"),
                     resample=r.updown)
        conv2 = dict(x=S["h1"], g=go, w=w2, y=S["out"], gamma=self.P(pre + "out_layers.0.weight"),
                     beta=self.P(pre + "out_layers.0.bias"), eps=GN_EPS, film=film, ld_film=self._E_ld,
                     bias=self.P(pre + "out_layers.3.bias"), **skip)
        # both launches planned with their exact arguments before the first is issued
        if not (ops.resconv_fwd(**conv1, query=True) and ops.resconv_fwd(**conv2, query=True)):
            return False
        p = self._pend
        self._pend = None
        ops.finalize(p)
        ok = ops.resconv_fwd(**conv1) and ops.resconv_fwd(**conv2)
        if not ok:
            raise RuntimeError("encdiff_resconv_fwd declined a conv its query with the same arguments accepted")
        return True

    def _res_fwd_agn(self, r: ResSpec, S, x, gi: Geom, go: Geom):
        """Inference ResBlock with its GroupNorms in the convs' A staging (EncdiffGemmArgs.agn_*):
        conv1 reads GN1+SiLU(x) (nearest-up through its gather), conv2 reads GN2+FiLM+SiLU(h1); no
        GroupNorm launch and no normalised activation in memory.  A down block keeps its GN1 launch
        (the conv reads the 2x2-averaged GroupNorm output).  Each conv combines its split-K slabs in
        the kernel, so its output is complete for the next conv's statistics."""
        pre = r.prefix
        if r.updown == L.RESAMPLE_DOWN2:
            ops.groupnorm_fwd(x, gi, self.P(pre + "in_layers.0.weight"), self.P(pre + "in_layers.0.bias"), S["a1"],
                              S["st1"], GN_EPS, True, in_stats=self._gst(x), x_from=self._take_pend(x))
            a1, rs = self._conv1_input(r, S, go)
            ops.conv3x3_fwd(a1, go, r.cin, self.W(pre + "in_layers.2.weight"), S["h1"],
                            bias=self.P(pre + "in_layers.2.bias"), resample=rs, fold=AGN_FOLD)
        else:
            p = self._pend  # x complete (a producer that deferred its finalize finalizes now)
            self._pend = None
            ops.finalize(p)
            ops.conv3x3_fwd(x, go, r.cin, self.W(pre + "in_layers.2.weight"), S["h1"],
                            bias=self.P(pre + "in_layers.2.bias"), resample=r.updown,
                            agn=(self.P(pre + "in_layers.0.weight"), self.P(pre + "in_layers.0.bias"), None, GN_EPS,
                                 True), fold=AGN_FOLD)
        out = S["out"]
        if r.cin != r.cout:
            ops.linear_fwd(x, self.W(pre + "skip_connection.weight"), out, bias=self.P(pre + "skip_connection.bias"))
            resid = out
        elif r.updown:
            ops.resample(x, S["xr"], go, r.updown)
            resid = S["xr"]
        else:
            resid = x
        film = self._E_use[:, r.film_off:]
        ops.conv3x3_fwd(S["h1"], go, r.cout, self.W(pre + "out_layers.3.weight"), out,
                        bias=self.P(pre + "out_layers.3.bias"), resid=resid, gn_stats=self._gst(out),
                        agn=(self.P(pre + "out_layers.0.weight"), self.P(pre + "out_layers.0.bias"), film, GN_EPS, True),
                        fold=AGN_FOLD)
        return out

    @staticmethod
    def _conv1_input(r: ResSpec, S, go: Geom):
        """in_layers conv input: the GN1 output, avg-pooled first for a down block
        (openaimodel_enc.py:256-261: in_rest -> h_upd -> in_conv) -- the pooled copy is
        kept for the weight gradient; nearest-up is read through the im2col gather."""
        if r.updown == L.RESAMPLE_DOWN2:
            ops.resample(S["a1"], S["a1r"], go, L.RESAMPLE_DOWN2)
            return S["a1r"], L.RESAMPLE_NONE
        return S["a1"], r.updown

    def _st_fwd(self, s: STSpec, x):
        """attention.py:250-261 (+ BasicTransformerBlock :211-215)."""
        B, c = self.B, s.c
        S = self.state[s.prefix]
        S["x"] = x
        g = Geom(B, s.h, s.h)
        tb = s.prefix + "transformer_blocks.0."
        ntok = s.h * s.h
        fused = ST_TAIL_FUSED and c <= ST_TAIL_MAXC and (self.infer or ST_TAIL_TRAIN)
        # the fused head: with the fused tail, or alone at inference for c = 256 sampling blocks
        hfused = fused or (ST_TAIL_FUSED and ST_HEAD_256 and self.infer and c == 256 and B <= ST_TAIL_HEAD_MAX_B)
        # inference, blocks whose LayerNorms would be launches of their own (c > 128: the GEMM
        # epilogue form needs the tile to span the row): norm1 / norm2 in the consumer's A staging
        lna = self.infer and LNA_IN and 128 < c <= 1024
        in_st = self._gst(x)
        # inference at sampling batches: the fused head computes the GroupNorm statistics itself
        self_st = hfused and in_st is None and self.infer and AGN and B <= AGN_MAX_B
        # x's producer deferred its split-K finalize: the unfused head's self-reducing GroupNorm
        # combines the slabs (and writes x); every other path reads x directly, so it is finalized now
        pend, self._pend = self._pend, None
        x_from = pend if (pend is not None and not hfused and in_st is None and pend.c == x.data_ptr()
                          and pend.N == x.shape[1] and pend.ldc == x.stride(0)) else None
        if x_from is None:
            ops.finalize(pend)
        if hfused and in_st is None and not self_st:  # no producer statistics: the GroupNorm kernel reduces them
            ops.groupnorm_fwd(x, g, self.P(s.prefix + "norm.weight"), self.P(s.prefix + "norm.bias"), S["gn"],
                              S["stg"], ST_GN_EPS, False)
        # GroupNorm (from producer statistics) + proj_in + norm1 + q/k/v as one kernel
        if not (hfused and ops.st_head_fwd(
                x, S["gn"], self.W(s.prefix + "proj_in.weight"), self.P(s.prefix + "proj_in.bias"),
                self.P(tb + "norm1.weight"), self.P(tb + "norm1.bias"), self.W(s.prefix + "qkv"), S["t0"], S["qkv"],
                B * ntok, c, ntok, ST_GN_EPS, LN_EPS, in_stats=in_st, gn_gamma=self.P(s.prefix + "norm.weight"),
                gn_beta=self.P(s.prefix + "norm.bias"), gn_stats=None if self_st else S["stg"],
                n1=None if self.infer else S["n1"], s1=None if self.infer else S["s1"], self_stats=self_st)):
            if not hfused or in_st is not None or self_st:
                ops.groupnorm_fwd(x, g, self.P(s.prefix + "norm.weight"), self.P(s.prefix + "norm.bias"), S["gn"],
                                  S["stg"], ST_GN_EPS, False, in_stats=in_st, x_from=x_from)
                x_from = None
            if lna:  # norm1 applied in q/k/v's A staging (no LayerNorm launch)
                ops.linear_fwd(S["gn"], self.W(s.prefix + "proj_in.weight"), S["t0"],
                               bias=self.P(s.prefix + "proj_in.bias"))
                ops.linear_fwd(S["t0"], self.W(s.prefix + "qkv"), S["qkv"],
                               ln_in=(self.P(tb + "norm1.weight"), self.P(tb + "norm1.bias"), LN_EPS))
            else:
                # proj_in, then norm1 in its epilogue (self-attention input)
                ops.linear_fwd_ln(S["gn"], self.W(s.prefix + "proj_in.weight"), S["t0"], self.P(tb + "norm1.weight"),
                                  self.P(tb + "norm1.bias"), S["n1"], S["s1"], LN_EPS,
                                  bias=self.P(s.prefix + "proj_in.bias"))
                ops.linear_fwd(S["n1"], self.W(s.prefix + "qkv"), S["qkv"])
        assert x_from is None, "a deferred finalize of the transformer input was neither combined nor run"
        q, k, v = S["qkv"][:, :c], S["qkv"][:, c:2 * c], S["qkv"][:, 2 * c:]
        ops.attention_fwd(q, k, v, S["o1"], S["lse1"], B, s.heads, ntok, ntok, s.dh, fp8=s.fp8)
        k2 = self.KV[:, s.kv_off:s.kv_off + c]
        v2 = self.KV[:, s.kv_off + c:s.kv_off + 2 * c]
        if (ST_TAIL_FUSED and ST_TAIL_C128_HEAD and not self.infer and c == 128
                and ops.st_tail_fwd(S["o1"], S["t0"], x, k2, v2, self._tail_weights(s), S["out"], B * ntok, c,
                                    ntok, s.heads, self.lu, LN_EPS, head=(S["t2"], S["n3"]),
                                    save={k: S[k] for k in ("t1", "n2", "q2", "o2", "t2", "n3", "s2", "s3", "lse2")})):
            return self._st_ff(s, x, S)
        if ST_TAIL_FUSED and c <= ST_TAIL_MAXC and (self.infer or ST_TAIL_TRAIN):
            save = None if self.infer else {k: S[k] for k in ("t1", "n2", "q2", "o2", "t2", "n3", "f", "a", "t3",
                                                             "s2", "s3")}
            if save is not None:
                save["lse2"] = S["lse2"]
            if ops.st_tail_fwd(S["o1"], S["t0"], x, k2, v2, self._tail_weights(s), S["out"], B * ntok, c, ntok,
                               s.heads, self.lu, LN_EPS, save=save, gn_stats=self._gst(S["out"]),
                               slots=self.stat_slots):
                return S["out"]
        if (ST_TAIL_FUSED and ST_TAIL_HEAD and self.infer and ST_TAIL_MAXC < c <= ST_TAIL_HEAD_MAXC
                and B <= ST_TAIL_HEAD_MAX_B
                and ops.st_tail_fwd(S["o1"], S["t0"], x, k2, v2, self._tail_weights(s), S["out"], B * ntok, c,
                                    ntok, s.heads, self.lu, LN_EPS, head=(S["t2"], S["n3"]))):
            return self._st_ff(s, x, S)
        if (ST_TAIL_FUSED and ST_TAIL_HEAD_TRAIN and not self.infer and ST_TAIL_MAXC < c <= ST_TAIL_HEAD_MAXC
                and ops.st_tail_fwd(S["o1"], S["t0"], x, k2, v2, self._tail_weights(s), S["out"], B * ntok, c,
                                    ntok, s.heads, self.lu, LN_EPS, head=(S["t2"], S["n3"]),
                                    save={k: S[k] for k in ("t1", "n2", "q2", "o2", "t2", "n3", "s2", "s3", "lse2")})):
            return self._st_ff(s, x, S)
        # cross-attention to the concept tokens (norm2 in the to_out epilogue, or at inference for
        # wide blocks in to_q's A staging)
        if lna:
            ops.linear_fwd(S["o1"], self.W(tb + "attn1.to_out.0.weight"), S["t1"],
                           bias=self.P(tb + "attn1.to_out.0.bias"), resid=S["t0"])
            ops.linear_fwd(S["t1"], self.W(tb + "attn2.to_q.weight"), S["q2"],
                           ln_in=(self.P(tb + "norm2.weight"), self.P(tb + "norm2.bias"), LN_EPS))
        else:
            ops.linear_fwd_ln(S["o1"], self.W(tb + "attn1.to_out.0.weight"), S["t1"], self.P(tb + "norm2.weight"),
                              self.P(tb + "norm2.bias"), S["n2"], S["s2"], LN_EPS,
                              bias=self.P(tb + "attn1.to_out.0.bias"), resid=S["t0"])
            ops.linear_fwd(S["n2"], self.W(tb + "attn2.to_q.weight"), S["q2"])
        ops.attention_fwd(S["q2"], k2, v2, S["o2"], S["lse2"], B, s.heads, ntok, self.lu, s.dh)
        # GEGLU feed-forward (norm3 in the to_out epilogue)
        ops.linear_fwd_ln(S["o2"], self.W(tb + "attn2.to_out.0.weight"), S["t2"], self.P(tb + "norm3.weight"),
                          self.P(tb + "norm3.bias"), S["n3"], S["s3"], LN_EPS,
                          bias=self.P(tb + "attn2.to_out.0.bias"), resid=S["t1"])
        return self._st_ff(s, x, S)

    def _st_ff(self, s: STSpec, x, S):
        """attention.py:215 + :260-261: the GEGLU feed-forward from n3 (residual t2), proj_out."""
        tb = s.prefix + "transformer_blocks.0."
        ops.linear_fwd_geglu(S["n3"], self.W(tb + "ff.net.0.proj.weight"), S["f"], S["a"],
                             bias=self.P(tb + "ff.net.0.proj.bias"))
        ops.linear_fwd(S["a"], self.W(tb + "ff.net.2.weight"), S["t3"], bias=self.P(tb + "ff.net.2.bias"),
                       resid=S["t2"])
        ops.linear_fwd(S["t3"], self.W(s.prefix + "proj_out.weight"), S["out"], bias=self.P(s.prefix + "proj_out.bias"),
                       resid=x, gn_stats=self._gst(S["out"]))
        return S["out"]

    def _tail_weights(self, s: STSpec):
        tb = s.prefix + "transformer_blocks.0."
        W, P = self.W, self.P
        return dict(out1=W(tb + "attn1.to_out.0.weight"), b_out1=P(tb + "attn1.to_out.0.bias"),
                    g2=P(tb + "norm2.weight"), be2=P(tb + "norm2.bias"), q2=W(tb + "attn2.to_q.weight"),
                    out2=W(tb + "attn2.to_out.0.weight"), b_out2=P(tb + "attn2.to_out.0.bias"),
                    g3=P(tb + "norm3.weight"), be3=P(tb + "norm3.bias"),
                    ff1=W(tb + "ff.net.0.proj.weight"), b_ff1=P(tb + "ff.net.0.proj.bias"),
                    ff2=W(tb + "ff.net.2.weight"), b_ff2=P(tb + "ff.net.2.bias"),
                    po=W(s.prefix + "proj_out.weight"), b_po=P(s.prefix + "proj_out.bias"))

    # ---------------------------------------------------------------- backward
    # ---------------------------------------------------------------- split backward (DP)
    @staticmethod
    def _early_final(name: str) -> bool:
        """Parameters whose gradient is complete once the output blocks' backward has run
        (the batched emb / cross-K/V / q,k,v weights are written later or live in the arena
        prefix, so they never count)."""
        n = name.split("diffusion_model.", 1)[-1]
        if not (n.startswith("output_blocks.") or n.startswith("out.")):
            return False
        return not any(k in n for k in (".emb_layers.1.", ".attn2.to_k.", ".attn2.to_v.", ".attn1.to_q.",
                                        ".attn1.to_k.", ".attn1.to_v."))

    @classmethod
    def arena_split_offset(cls, arena: ParamArena, names: Sequence[str]) -> Optional[int]:
        """Arena offset where the output-block / out parameters begin, when every other UNet
        parameter of `names` ends before it (None otherwise)."""
        span = {}
        for n in names:
            o, sh = arena.offsets[n]
            span[n] = (o, o + int(torch.Size(sh).numel()))
        early = [n for n in names if cls._early_final(n)]
        if not early:
            return None
        lo = min(span[n][0] for n in early)
        if any(span[n][1] > lo for n in names if not cls._early_final(n)):
            return None
        return lo

    def split_plan(self, names: Sequence[str]) -> Optional[int]:
        """For data-parallel overlap: the arena offset `lo` such that [lo, end of the UNet
        parameters) holds exactly the output-block / out parameters (their gradients are final
        after `backward(split=True)`, and can be all-reduced while `backward_rest` runs), and
        the GroupNorm / LayerNorm partial columns of those layers form suffixes.  None when the
        layout does not allow it (the caller then runs the backward unsplit)."""
        if getattr(self, "_split", False) is not False:
            return self._split[0] if self._split else None
        self._split = None
        lo = self.arena_split_offset(self.arena, names)
        if lo is None:
            return None
        gcol = self.gn.split_col(self._early_final)
        lcol = self.ln.split_col(self._early_final)
        fcol = self.ln_f.split_col(self._early_final)
        if gcol is None or lcol is None or fcol is None:
            return None
        self._split = (lo, gcol, lcol, fcol)
        return lo

    def backward(self, d_eps: torch.Tensor, split: bool = False) -> torch.Tensor:
        """d_eps (B,C,H,W) fp32 -> d_context (B, latent_unit*context_dim) fp32.  Accumulates
        every UNet weight gradient into the arena (which the caller zeroed).

        split=True (data-parallel overlap, needs a successful `split_plan`): stop after the
        output blocks with their gradients final in the arena; `backward_rest()` then runs the
        middle / input blocks and the batched emb / K,V GEMMs and fills the returned d_context
        buffer.  Launch for launch the same work as the unsplit backward (the last deferred
        finalize and the norm partial fold are issued in two parts)."""
        ops.group_begin(self._wgg if ops.WG_GROUP else None)
        self._wg_blocks = 0
        try:
            out = self._bwd_outputs(d_eps)
            if split and self._split:
                ops.group_end()  # the output blocks' weight gradients, one grid
                _, gcol, lcol, fcol = self._split
                ops.flush()
                self.gn.reduce(gcol)
                self.ln.reduce(lcol)
                self.ln_f.reduce(fcol)
                self._cont = out
                return self.d_ctx
            self._cont = None
            return self._bwd_rest(out, self.gn.cols, self.ln.cols, self.ln_f.cols)
        finally:
            ops.group_begin(None)

    def _wg_block_done(self):
        """A UNet block's backward is issued: every WG_WINDOW blocks the collected weight gradients
        run as one grid while their operands are hot."""
        self._wg_blocks += 1
        if WG_WINDOW > 0 and self._wg_blocks % WG_WINDOW == 0:
            ops.group_flush()

    def backward_rest(self) -> torch.Tensor:
        assert self._cont is not None, "backward_rest() follows backward(split=True)"
        out, self._cont = self._cont, None
        _, gcol, lcol, fcol = self._split
        self._wg_blocks = 0
        ops.group_begin(self._wgg if ops.WG_GROUP else None)
        try:
            return self._bwd_rest(out, gcol, lcol, fcol)
        finally:
            ops.group_begin(None)

    def _bwd_outputs(self, d_eps: torch.Tensor):
        B = self.B
        sp = self.spec
        g0 = Geom(B, self.H, self.H)
        d_eps = d_eps.contiguous()
        # out conv (mc -> 3): input gradient on the VALU kernel; weight gradient as a GEMM over
        # channel-padded d eps rows (rows 3..7 zero), folded into the reference layout; bias = sum
        ops.small_conv_out_bwd(self.a_out, g0, self.P("out.2.weight"), d_eps, self.d_aout, None, None)
        ops.nchw_to_rows(d_eps, 8, self.deps8)
        co = d_eps.shape[1]
        # bias gradient = column sums of the padded d eps rows (the GEMM's bias-gradient
        # accumulator db_out, emptied by the fold)
        ops.gemm(8, 9 * sp.out_ch, g0.pixels, self.deps8, 8, self.a_out, self.a_out.stride(0), self.dw_out,
                 9 * sp.out_ch, a_mode=L.OPA_ROWM, b_mode=L.OPB_IM2COL, c_mode=L.OUT_F32,
                 conv=L.ConvGeom(batch=B, h=self.H, w=self.H, cin=sp.out_ch, resample=0,
                                 ld_src=self.a_out.stride(0)), bias_grad=self.db_out)
        ops.grad_fold(self.dw_out, co, sp.out_ch, sp.out_ch, 9, self.G("out.2.weight"), self.db_out,
                      self.G("out.2.bias"))
        dg, db = self.gn.parts("out.0.weight", sp.out_ch)
        ops.groupnorm_bwd(self._h_last, g0, self.P("out.0.weight"), self.P("out.0.bias"), self.st_out, GN_EPS, True,
                          self.d_aout, self.d_hlast, dg, db, ld_part=self.gn.ld, dsilu=self.ds_out)
        dout = self.d_hlast
        hs = self._hs
        nhs = len(hs)
        g_hs: List[Optional[torch.Tensor]] = [None] * nhs
        for j in range(len(sp.output_blocks) - 1, -1, -1):
            blk = sp.output_blocks[j]
            for li in range(len(blk) - 1, -1, -1):
                layer = blk[li]
                if li == 0:
                    dx_target, acc = self.dxcat[j], False
                else:
                    dx_target, acc = self.state[layer.prefix]["d_in"], False
                self._layer_bwd(layer, dout, dx_target, acc)
                dout = dx_target
            c1 = blk[0].cin - sp.skip_ch[nhs - 1 - j]
            g_hs[nhs - 1 - j] = self.dxcat[j][:, c1:]
            dout = self.dxcat[j][:, :c1]
            self._wg_block_done()
        return dout, g_hs

    def _bwd_rest(self, state, gcol: int, lcol: int, fcol: int) -> torch.Tensor:
        B = self.B
        sp = self.spec
        g0 = Geom(B, self.H, self.H)
        dout, g_hs = state
        nhs = len(self._hs)
        # middle block: its input is hs[-1]
        for li in range(len(sp.middle) - 1, -1, -1):
            layer = sp.middle[li]
            if li == 0:
                dx_target, acc = g_hs[nhs - 1], True
            else:
                dx_target, acc = self.state[layer.prefix]["d_in"], False
            self._layer_bwd(layer, dout, dx_target, acc)
            dout = dx_target
        self._wg_block_done()
        # input blocks 11..1: output grad = g_hs[i] (complete), input grad accumulates into g_hs[i-1]
        for i in range(len(sp.input_blocks) - 1, 0, -1):
            blk = sp.input_blocks[i]
            dout = g_hs[i]
            for li in range(len(blk) - 1, -1, -1):
                layer = blk[li]
                if li == 0:
                    dx_target, acc = g_hs[i - 1], True
                else:
                    dx_target, acc = self.state[layer.prefix]["d_in"], False
                self._layer_bwd(layer, dout, dx_target, acc)
                dout = dx_target
            self._wg_block_done()
        # input conv weight grad (no input grad: x_t carries no gradient)
        dy0 = g_hs[0]
        ops.gemm(self.mc, 72, g0.pixels, dy0, dy0.stride(0), self.x8, 8, self.dw_in, 72, a_mode=L.OPA_ROWM,
                 b_mode=L.OPB_IM2COL, c_mode=L.OUT_F32,
                 conv=L.ConvGeom(batch=B, h=self.H, w=self.H, cin=8, resample=0, ld_src=8),
                 bias_grad=self.G("input_blocks.0.0.bias"))
        cin0 = self._x.shape[1]
        ops.grad_fold(self.dw_in, self.mc, cin0, 8, 9, self.G("input_blocks.0.0.weight"))
        if self.want_dx:
            # d x_t (only when the caller asked for it: the EncDiff objective needs none): the
            # input conv's input gradient over the channel-padded rows, fp32, back to NCHW
            if getattr(self, "d_x", None) is None or self.d_x.shape != self._x.shape:
                self.dx8 = torch.empty(g0.pixels, 8, device=self.dev, dtype=F32)
                self.d_x = torch.empty_like(self._x, dtype=F32)
            ops.gemm(g0.pixels, 8, 9 * self.mc, dy0, dy0.stride(0), self.W("input_conv"), 72, self.dx8, 8,
                     a_mode=L.OPA_IM2COL, b_mode=L.OPB_CONV_DGRAD, c_mode=L.OUT_F32,
                     conv=L.ConvGeom(batch=B, h=self.H, w=self.H, cin=self.mc, resample=0, ld_src=dy0.stride(0)),
                     conv_cout=self.mc)
            ops.nchw_rows_f32(self.dx8, B, cin0, self.H * self.H, 8, self.d_x, 8, to_rows=False)
        # batched emb_layers backward -> time MLP
        ops.ew(L.EW_F32_TO_BF16, self.dE, self.dE16)
        ops.linear_bwd(self.dE16, self.W("emb_all"), self.emb_s, self.d_emb_s, self.emb_w_grad, self.emb_bias_grad)
        ops.ew(L.EW_SILU_BWD, self.emb, self.d_emb, x2=self.d_emb_s)
        ops.linear_bwd(self.d_emb, self.W("time_embed.2.weight"), self.ta1, self.d_ta1, self.G("time_embed.2.weight"),
                       self.G("time_embed.2.bias"))
        ops.ew(L.EW_SILU_BWD, self.th1, self.d_th1, x2=self.d_ta1)
        ops.linear_wgrad(self.d_th1, self.temb0, self.G("time_embed.0.weight"), self.G("time_embed.0.bias"))
        # batched cross-attention K/V backward -> context gradient (fp32 output: separate GEMM)
        ops.gemm(B * self.lu, self.cd, sp.kv_total, self.dKV, self.dKV.stride(0), self.W("kv_all"), self.cd,
                 self.d_ctx, self.cd, b_mode=L.OPB_ROWN, c_mode=L.OUT_F32)
        ops.linear_wgrad(self.dKV, self.ctx16, self.kv_w_grad)
        ops.group_end()  # every weight gradient since group_begin, one grid
        ops.flush()  # the last deferred weight-gradient finalize (paired launches)
        # fold the norm affine partial sums into the arena (all of them, or what the split
        # backward left: the columns before the output blocks' suffix)
        self.gn.reduce(0, gcol)
        self.ln.reduce(0, lcol)
        self.ln_f.reduce(0, fcol)
        return self.d_ctx

    def conv_bwd(self, dy, g, cin, name, x, dx, db, resample=0, defer_dx=False):
        """Backward of a 3x3 conv (weight `name`): weight and input gradient in one launch.
        defer_dx: returns the input gradient's GemmArgs when its split-K finalize was left to
        the GroupNorm backward that reads dx (groupnorm_bwd(dy_from=...)), else None."""
        if name in self.arena.cl:
            return ops.conv3x3_bwd_cl(dy, g, self.W(name), x, cin, self.arena.raw(self.arena.grad, name), dx, db,
                                      resample=resample, defer_dx=defer_dx)
        ops.conv3x3_dgrad(dy, g, self.W(name), dx)
        self.conv_wgrad(dy, x, g, cin, name, db, resample=resample)
        return None

    def _layer_bwd(self, layer, dout, dx, acc):
        if isinstance(layer, ResSpec):
            self._res_bwd(layer, dout, dx, acc)
        else:
            self._st_bwd(layer, dout, dx, acc)

    def _res_bwd(self, r: ResSpec, dout, dx, acc):
        B = self.B
        S = self.state[r.prefix]
        x = S["x"]
        gi, go = Geom(B, r.hin, r.hin), Geom(B, r.hout, r.hout)
        pre = r.prefix
        # conv2: input + weight gradient in one launch
        # (the input gradients' split-K finalizes ride in the GroupNorm backwards that read them)
        f2 = self.conv_bwd(dout, go, r.cout, pre + "out_layers.3.weight", S["a2"], S["d_a2"],
                           self.G(pre + "out_layers.3.bias"), defer_dx=GN_FIN)
        # GN2 + FiLM + SiLU
        dg, db = self.gn.parts(pre + "out_layers.0.weight", r.cout)
        ops.groupnorm_bwd(S["h1"], go, self.P(pre + "out_layers.0.weight"), self.P(pre + "out_layers.0.bias"),
                          S["st2"], GN_EPS, True, S["d_a2"], S["d_h1"], dg, db, film=self.E[:, r.film_off:],
                          ld_film=self.E.shape[1], dfilm=self.dE[:, r.film_off:], ld_dfilm=self.dE.shape[1],
                          ld_part=self.gn.ld, dy_from=f2, dsilu=S.get("ds2"))
        # conv1 (on the resampled GN1 output)
        if r.updown == L.RESAMPLE_DOWN2:
            a1, rs = S["a1r"], L.RESAMPLE_NONE
        else:
            a1, rs = S["a1"], r.updown
        dg, db = self.gn.parts(pre + "in_layers.0.weight", r.cin)
        d_a1 = S["d_a1"]
        f1 = self.conv_bwd(S["d_h1"], go, r.cin, pre + "in_layers.2.weight", a1, S["d_a1r"] if r.updown else d_a1,
                           self.G(pre + "in_layers.2.bias"), resample=rs, defer_dx=GN_FIN and not r.updown)
        fuse = RS_FUSED and r.updown and r.cin == r.cout
        if r.updown and not fuse:
            ops.resample_bwd(S["d_a1r"], d_a1, gi, r.updown)
        identity = r.cin == r.cout and not r.updown
        # identity skip: its gradient (dout) rides in the GN1 backward pass; so do, for a resampling
        # block, the resample adjoints of conv1's input gradient and of the skip branch
        ops.groupnorm_bwd(x, gi, self.P(pre + "in_layers.0.weight"), self.P(pre + "in_layers.0.bias"), S["st1"],
                          GN_EPS, True, S["d_a1r"] if fuse else d_a1, dx, dg, db, accumulate=acc, ld_part=self.gn.ld,
                          resid=dout if (identity or fuse) else None, dy_from=f1,
                          dy_resample=r.updown if fuse else 0, resid_resample=r.updown if fuse else 0,
                          dsilu=S.get("ds1"))
        # skip path
        if r.cin != r.cout:
            ops.linear_bwd(dout, self.W(pre + "skip_connection.weight"), x, dx,
                           self.G(pre + "skip_connection.weight").view(r.cout, r.cin),
                           self.G(pre + "skip_connection.bias"), resid=dx)
        elif r.updown and not fuse:
            ops.resample_bwd(dout, dx, gi, r.updown, accumulate=True)

    def _st_bwd_fused(self, s: STSpec, dout, dx, acc) -> bool:
        """attention.py:250-261 backward in 5 launches: the tail's input-gradient chain
        (encdiff_st_tail_bwd: proj_out, GEGLU FF, norm3, attn2 with its cross-attention backward,
        norm2, attn1.to_out), the self-attention backward, the head's chain (encdiff_st_head_bwd:
        q/k/v, norm1, proj_in), the block's 8 weight gradients as one grouped launch, and the
        GroupNorm backward with the block residual.  False (nothing launched): shape outside the
        fused kernels' support -- the caller runs the per-layer launches."""
        B, c = self.B, s.c
        S = self.state[s.prefix]
        x = S["x"]
        tb = s.prefix + "transformer_blocks.0."
        ntok = s.h * s.h
        X = self.st_scratch[(s.h, c)]
        W, P, G = self.W, self.P, self.G
        wt = {k: W(s.prefix + "T:" + k) for k in ("po", "ff2", "ff1", "out2", "q2", "out1")}
        k2 = self.KV[:, s.kv_off:s.kv_off + c]
        v2 = self.KV[:, s.kv_off + c:s.kv_off + 2 * c]
        dk2 = self.dKV[:, s.kv_off:s.kv_off + c]
        dv2 = self.dKV[:, s.kv_off + c:s.kv_off + 2 * c]
        save = {k: S[k] for k in ("f", "t2", "t1", "q2", "o2", "s3", "s2", "lse2")}
        out = dict(d_t3=S["d_t3"], d_f=S["d_f"], d_t2=S["d_t2"], d_q2=S["d_q2"], d_t1=S["d_t1"], d_o1=X["d_o"])
        F = self.ln_f
        if not ops.st_tail_bwd(dout, save, wt, P(tb + "norm3.weight"), P(tb + "norm2.weight"), k2, v2, out,
                               F.parts(tb + "norm3.weight", c), F.parts(tb + "norm2.weight", c), dk2, dv2,
                               B * ntok, c, ntok, s.heads, self.lu, kv_part=X["kv_part"]):
            return False
        tiles = ntok // ops.st_tail_bwd_tile(c, B * ntok, ntok)  # per image: > 1 -> partial slabs
        qkv, dqkv = S["qkv"], S["d_qkv"]
        ops.attention_bwd(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], S["o1"], S["lse1"], X["d_o"], dqkv[:, :c],
                          dqkv[:, c:2 * c], dqkv[:, 2 * c:], B, s.heads, ntok, ntok, s.dh, fp8=s.fp8)
        ok = ops.st_head_bwd(dqkv, S["d_t1"], S["t0"], S["s1"], P(tb + "norm1.weight"), W(s.prefix + "T:qkv"),
                             W(s.prefix + "T:in"), S["d_t0"], X["d_g"], F.parts(tb + "norm1.weight", c), B * ntok, c,
                             kv=(X["kv_part"], tiles, self.lu, B, dk2, dv2) if tiles > 1 else None)
        if not ok:
            raise RuntimeError("encdiff_st_head_bwd declined a block whose tail it accepted")
        wg = [(dout, S["t3"], G(s.prefix + "proj_out.weight").view(c, c), G(s.prefix + "proj_out.bias")),
              (S["d_t3"], S["a"], G(tb + "ff.net.2.weight"), G(tb + "ff.net.2.bias")),
              (S["d_f"], S["n3"], G(tb + "ff.net.0.proj.weight"), G(tb + "ff.net.0.proj.bias")),
              (S["d_t2"], S["o2"], G(tb + "attn2.to_out.0.weight"), G(tb + "attn2.to_out.0.bias")),
              (S["d_q2"], S["n2"], G(tb + "attn2.to_q.weight"), None),
              (S["d_t1"], S["o1"], G(tb + "attn1.to_out.0.weight"), G(tb + "attn1.to_out.0.bias")),
              (dqkv, S["n1"], self.qkv_grad[s.prefix], None),
              (S["d_t0"], S["gn"], G(s.prefix + "proj_in.weight").view(c, c), G(s.prefix + "proj_in.bias"))]
        fold = None
        if ST_BWD_WG == "st":
            # (slabs in a scratch of their own: a paired launch's deferred finalize stays pending)
            fold = self._stwgk.launch(wg, ride=ST_FOLD_RIDE)
        elif ST_BWD_WG == "group":
            ops.flush()
            for dy_, x_, dw, db in wg:
                self._stwg.add(ops.whole_wgrad_args(dy_, x_, dw, db))
            self._stwg.launch()
        else:
            for dy_, x_, dw, db in wg:
                ops.linear_wgrad(dy_, x_, dw, db)
        dg, db = self.gn.parts(s.prefix + "norm.weight", c)
        ops.groupnorm_bwd(x, Geom(B, s.h, s.h), P(s.prefix + "norm.weight"), P(s.prefix + "norm.bias"), S["stg"],
                          ST_GN_EPS, False, X["d_g"], dx, dg, db, accumulate=acc, ld_part=self.gn.ld, resid=dout,
                          fold=fold)
        return True

    def _st_bwd(self, s: STSpec, dout, dx, acc):
        if s.prefix in self.stf:
            if self._st_bwd_fused(s, dout, dx, acc):
                return
            raise RuntimeError(f"encdiff_st_tail_bwd declined {s.prefix} (c={s.c}, {s.h}x{s.h}, B={self.B})")
        B, c = self.B, s.c
        S = self.state[s.prefix]
        x = S["x"]
        g = Geom(B, s.h, s.h)
        tb = s.prefix + "transformer_blocks.0."
        ntok = s.h * s.h
        X = self.st_scratch[(s.h, c)]
        d_a, d_n, d_o = X["d_a"], X["d_n"], X["d_o"]
        # proj_out
        d_t3 = S["d_t3"]
        ops.linear_bwd(dout, self.W(s.prefix + "proj_out.weight"), S["t3"], d_t3,
                       self.G(s.prefix + "proj_out.weight").view(c, c), self.G(s.prefix + "proj_out.bias"))
        # FF
        ops.linear_bwd_geglu(d_t3, self.W(tb + "ff.net.2.weight"), S["a"], S["f"], S["d_f"],
                             self.G(tb + "ff.net.2.weight"), self.G(tb + "ff.net.2.bias"), d_a=d_a)
        fin = ops.linear_bwd(S["d_f"], self.W(tb + "ff.net.0.proj.weight"), S["n3"], d_n,
                             self.G(tb + "ff.net.0.proj.weight"), self.G(tb + "ff.net.0.proj.bias"), defer_dx=GN_FIN)
        dg, db = self.ln.parts(tb + "norm3.weight", c)
        d_t2 = S["d_t2"]  # d(t2) = d(t3) (residual) + norm3 backward
        ops.layernorm_bwd(S["t2"], self.P(tb + "norm3.weight"), S["s3"], d_n, d_t2, dg, db, ld_part=self.ln.ld,
                          resid=d_t3, dy_from=fin)
        # cross-attention
        ops.linear_bwd(d_t2, self.W(tb + "attn2.to_out.0.weight"), S["o2"], d_o,
                       self.G(tb + "attn2.to_out.0.weight"), self.G(tb + "attn2.to_out.0.bias"))
        k2 = self.KV[:, s.kv_off:s.kv_off + c]
        v2 = self.KV[:, s.kv_off + c:s.kv_off + 2 * c]
        dk2 = self.dKV[:, s.kv_off:s.kv_off + c]
        dv2 = self.dKV[:, s.kv_off + c:s.kv_off + 2 * c]
        ops.attention_bwd(S["q2"], k2, v2, S["o2"], S["lse2"], d_o, S["d_q2"], dk2, dv2, B, s.heads, ntok, self.lu,
                          s.dh)
        fin = ops.linear_bwd(S["d_q2"], self.W(tb + "attn2.to_q.weight"), S["n2"], d_n,
                             self.G(tb + "attn2.to_q.weight"), defer_dx=GN_FIN)
        dg, db = self.ln.parts(tb + "norm2.weight", c)
        d_t1 = S["d_t1"]
        ops.layernorm_bwd(S["t1"], self.P(tb + "norm2.weight"), S["s2"], d_n, d_t1, dg, db, ld_part=self.ln.ld,
                          resid=d_t2, dy_from=fin)
        # self-attention
        ops.linear_bwd(d_t1, self.W(tb + "attn1.to_out.0.weight"), S["o1"], d_o,
                       self.G(tb + "attn1.to_out.0.weight"), self.G(tb + "attn1.to_out.0.bias"))
        qkv, dqkv = S["qkv"], S["d_qkv"]
        ops.attention_bwd(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], S["o1"], S["lse1"], d_o, dqkv[:, :c],
                          dqkv[:, c:2 * c], dqkv[:, 2 * c:], B, s.heads, ntok, ntok, s.dh, fp8=s.fp8)
        fin = ops.linear_bwd(dqkv, self.W(s.prefix + "qkv"), S["n1"], d_n, self.qkv_grad[s.prefix], defer_dx=GN_FIN)
        dg, db = self.ln.parts(tb + "norm1.weight", c)
        d_t0 = S["d_t0"]
        ops.layernorm_bwd(S["t0"], self.P(tb + "norm1.weight"), S["s1"], d_n, d_t0, dg, db, ld_part=self.ln.ld,
                          resid=d_t1, dy_from=fin)
        # proj_in
        fin = ops.linear_bwd(d_t0, self.W(s.prefix + "proj_in.weight"), S["gn"], X["d_g"],
                             self.G(s.prefix + "proj_in.weight").view(c, c), self.G(s.prefix + "proj_in.bias"),
                             defer_dx=GN_FIN)
        dg, db = self.gn.parts(s.prefix + "norm.weight", c)
        # + the residual x_in branch (dout), in the same pass (and proj_in's input-gradient finalize)
        ops.groupnorm_bwd(x, g, self.P(s.prefix + "norm.weight"), self.P(s.prefix + "norm.bias"), S["stg"], ST_GN_EPS,
                          False, X["d_g"], dx, dg, db, accumulate=acc, ld_part=self.gn.ld, resid=dout, dy_from=fin)
