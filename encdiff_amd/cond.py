"""HIP executor of the concept encoder's convolution trunk.

Encoder4.encoder (openaimodel_enc.py:996-1012) is

    Conv2d(3, d, 4, 2, 1)  BN ReLU      64x64 -> 32x32   (image_size 128: one more [Conv BN ReLU])
    Conv2d(d, d, 4, 2, 1)  BN ReLU            -> 16x16
    Conv2d(d, d, 4, 2, 1)  BN                 ->  8x8
    Conv2d(d, d, 4, 2, 1)  BN ReLU            ->  4x4
    EncResBlock(bn)  BN ReLU  EncResBlock(bn)       (x + conv1x1(ReLU(BN(conv3x3(ReLU(x))))))
    View(-1, d*16)  Linear(d*16, latent_unit)

trained with batch statistics.  The reference runs it in fp32 through cuDNN/MIOpen
(~60 launches, ~1.9 ms per fwd+bwd at B=128 on the MI355X).  Here the convolutions are
the UNet's implicit-im2col MFMA GEMMs (Conv2d(k4,s2,p1) is an im2col mode; its input
gradient the transposed mode; each layer's input and weight gradients one paired launch),
BatchNorm+ReLU are two launches each way (deterministic last-workgroup folds), and
activations are NHWC: bf16 GEMM operands, fp32 pre-BatchNorm tensors (conv outputs and the
residual sums), so the batch statistics and the ReLU masks are taken on fp32 values as in
the reference.  Both EncResBlock inputs are ReLU outputs, so their leading
ReLU is the identity and its gradient mask equals the preceding BN-ReLU's (mask^2 = mask).
The trunk hands its output to the reference modules as the fp32 NCHW-flattened
(B, d*16) tensor, so `Linear(d*16, latent_unit)` and the warp MLPs follow unchanged.

Forward precision (bf16x3).  Four BatchNorm+ReLU stages sit between the image and the
trunk's output, so the backward's ReLU masks are as good as the forward's pre-BN values.  Plain
bf16 operands (fp32 accumulation) move ~0.2 % of those values across zero, which shows as
~13 % rel-L2 in the first convolutions' weight gradients against the fp32 reference (measured
on the GPU and reproduced by a CPU emulation; split-bf16 operands: 0.5 %).  So every forward
GEMM of the trunk runs on split-bf16 operands, v = hi + lo with hi = bf16(v), lo = bf16(v - hi):
activations are stored as [hi | lo | hi] channel blocks (written by the BatchNorm apply / image
repack), weights packed [hi | hi | lo] (PackJob kinds 3-5), and ONE GEMM over K' = 3K forms
a_hi w_hi + a_lo w_hi + a_hi w_lo -- ~16 significant bits per product.  The EncResBlock 1x1 conv
also takes its residual input as [h_hi | h_lo] blocks against identity weights, so the residual
sum is formed in fp32 inside the same GEMM.  The backward stays bf16 (hi blocks, hi weights):
gradient rounding does not move masks.

Weight gradients are written into the fp32 parameter arena (the modules' .grad views);
only d(input image) is not computed (the image carries no gradient).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List

import torch

from . import _lib as L
from . import ops
from .arena import PackTable
from .ops import Geom

BF16 = torch.bfloat16
F32 = torch.float32


class _Conv:
    def __init__(self, name: str, mod: torch.nn.Conv2d, hout: int, k4: bool):
        self.name, self.mod, self.hout, self.k4 = name, mod, hout, k4
        self.cout, self.cin = mod.weight.shape[0], mod.weight.shape[1]


class Encoder4TrunkExecutor:
    """Binds Encoder4.encoder (all but View + Linear) to the parameter arena."""

    @staticmethod
    def layout(enc):
        """Walk Encoder4.encoder (openaimodel_enc.py:996-1013; any number of stride-2 stages,
        see Encoder4's image_size): [(conv idx, bn idx, relu)] for the Conv2d(k4, s2, p1) stages,
        [(res idx, post-bn idx or None)] for the two EncResBlocks, the Linear's index."""
        mods = list(enc.encoder)
        stages, res, lin = [], [], None
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, torch.nn.Conv2d):
                assert m.kernel_size == (4, 4) and m.stride == (2, 2) and isinstance(mods[i + 1], torch.nn.BatchNorm2d)
                relu = i + 2 < len(mods) and isinstance(mods[i + 2], torch.nn.ReLU)
                stages.append((i, i + 1, relu))
                i += 3 if relu else 2
            elif type(m).__name__ == "EncResBlock":
                post = i + 1 if isinstance(mods[i + 1], torch.nn.BatchNorm2d) else None
                res.append((i, post))
                i += 3 if post is not None else 1
            elif isinstance(m, torch.nn.Linear):
                lin = i
                i += 1
            else:
                i += 1
        assert len(res) == 2 and lin == len(mods) - 1 and len(stages) >= 2, "Encoder4 trunk layout"
        return stages, res, lin

    def __init__(self, enc, arena, prefix: str):
        seq = enc.encoder
        self.enc = enc
        self.arena = arena
        self.prefix = prefix
        self.dev = arena.device
        mods = list(seq)
        stages, res, lin = self.layout(enc)
        self.d = mods[0].weight.shape[0]
        self.cin_img = mods[0].weight.shape[1]
        assert self.cin_img <= 8, "Encoder4 trunk layout"
        self.img = 4 << len(stages)  # input resolution: every stage halves, the last output is 4x4
        hs = [self.img >> (k + 1) for k in range(len(stages))]
        self.convs = [_Conv(f"encoder.{ci}", mods[ci], h, True) for (ci, _, _), h in zip(stages, hs)]
        self.bns = [(f"encoder.{bi}", mods[bi], r) for _, bi, r in stages]
        self.res = []
        for ri, bi in res:
            rb = mods[ri]
            c3, bnm, c1 = rb.convs[1], rb.convs[2], rb.convs[4]
            self.res.append(dict(prefix=f"encoder.{ri}.convs.", conv3=c3, bn=bnm, conv1=c1,
                                 post_bn=(f"encoder.{bi}", mods[bi]) if bi is not None else None))
        self.flat = mods[lin]
        self.lin_name = f"encoder.{lin}"
        pk = PackTable(arena)
        a = arena
        c0 = self.convs[0]
        d = self.d
        # bf16 weights of the backward (input gradients) ...
        # first conv: [d][3][4][4] -> [d][16 taps][8] (channels padded with zeros)
        pk.add("c0", a.offsets[self.pn(c0.name + ".weight")][0], d, 16 * 8, kind=2, cin=self.cin_img)
        for c in self.convs[1:]:
            pk.add(c.name, a.offsets[self.pn(c.name + ".weight")][0], c.cout, 16 * c.cin)
        for r in self.res:
            p = r["prefix"]
            pk.add(p + "1", a.offsets[self.pn(p + "1.weight")][0], d, 9 * d)
            pk.add(p + "4", a.offsets[self.pn(p + "4.weight")][0], d, d)
        # ... and the split-bf16 [hi|hi|lo] weights of the forward (bf16x3, see the module doc)
        pk.add("c0x3", a.offsets[self.pn(c0.name + ".weight")][0], d, 16 * 24, kind=4, cin=self.cin_img)
        for c in self.convs[1:]:
            pk.add(c.name + "x3", a.offsets[self.pn(c.name + ".weight")][0], c.cout, 16 * 3 * c.cin, kind=3,
                   cin=c.cin)
        for r in self.res:
            p = r["prefix"]
            pk.add(p + "1x3", a.offsets[self.pn(p + "1.weight")][0], d, 9 * 3 * d, kind=3, cin=d)
            pk.add(p + "4x5", a.offsets[self.pn(p + "4.weight")][0], d, 5 * d, kind=5, cin=d)
        pk.finalize()
        pk.repack()
        self.pack = pk
        self._bufs: Dict[int, dict] = {}
        self._nbt = None
        self._bind_counters()

    def _bind_counters(self):
        """The trunk's BatchNorm2d.num_batches_tracked buffers become views of ONE int64 tensor, so
        a training forward advances all of them with one launch (BatchNorm2d.train() semantics,
        state_dict parity) instead of one torch kernel per module.  Rebound if the module moved
        its buffers (e.g. .to())."""
        mods = [m for _, m, _ in self.bns] + [r["bn"] for r in self.res] + \
               [r["post_bn"][1] for r in self.res if r["post_bn"] is not None]
        mods = [m for m in mods if m.num_batches_tracked is not None]
        if not mods:
            return
        shared = torch.stack([m.num_batches_tracked.detach().to(self.dev) for m in mods])
        for i, m in enumerate(mods):
            m._buffers["num_batches_tracked"] = shared[i]
        self._nbt, self._nbt_mods = shared, mods

    def _count_batch(self):
        if self._nbt is None:
            return
        m0 = self._nbt_mods[0]
        if m0.num_batches_tracked.data_ptr() != self._nbt.data_ptr():
            self._bind_counters()
        self._nbt.add_(1)

    # ------------------------------------------------------------ helpers
    def pn(self, local: str) -> str:
        return self.prefix + local

    def P(self, local):
        return self.arena.f32(self.pn(local))

    def G(self, local):
        return self.arena.grad_of(self.pn(local))

    def Graw(self, local):
        return self.arena.raw(self.arena.grad, self.pn(local))

    @classmethod
    def channels_last_names(cls, enc, prefix: str) -> List[str]:
        """Conv weights the arena stores [co][kh][kw][ci] (the GEMM B layout): every stride-2
        conv but the first (image channels padded to 8 in its own pack) and the EncResBlocks'
        3x3 convs."""
        stages, res, _ = cls.layout(enc)
        out = [prefix + f"encoder.{ci}.weight" for ci, _, _ in stages[1:]]
        out += [prefix + f"encoder.{ri}.convs.1.weight" for ri, _ in res]
        return out

    def _bn_state(self, B, key, rows, c):
        bufs = self._bufs[B]
        st = bufs.get("bn:" + key)
        if st is None:
            n = L.lib.encdiff_batchnorm_partials_floats(rows, c)
            st = bufs["bn:" + key] = dict(mean=torch.empty(c, device=self.dev), rstd=torch.empty(c, device=self.dev),
                                          part=torch.empty(n, device=self.dev),
                                          counter=torch.zeros(1, device=self.dev, dtype=torch.int32))
        return st

    def _bind(self, B):
        if B in self._bufs:
            return self._bufs[B]
        t = lambda rows, c, dt=BF16: torch.empty(rows, c, device=self.dev, dtype=dt)  # noqa: E731
        d = self.d
        # forward GEMM operands are split-bf16 rows [hi | lo | hi]; pre-BatchNorm tensors (conv
        # outputs, residual sums) are fp32 (see the module doc)
        b = dict(x0=t(B * self.img * self.img, 24))
        for i, c in enumerate(self.convs):
            n = B * c.hout * c.hout
            b[f"c{i}"], b[f"dc{i}"], b[f"da{i}"] = t(n, d, F32), t(n, d), t(n, d)
            if i < len(self.convs) - 1:
                b[f"a{i}"] = t(n, 3 * d)
        n4 = B * 16
        for j in range(2):
            # res block j operand rows: [u_hi u_lo u_hi | h_hi h_lo h_hi] -- the 3x3 conv reads the
            # h blocks, the 1x1 conv + identity residual the first five
            b[f"R{j}"] = t(n4, 6 * d)
            for k in ("t", "r", "dt", "du", "dr", "dh"):
                b[f"{k}{j}"] = t(n4, d, F32 if k in ("t", "r") else BF16)
        b["dw0"] = t(d, 16 * 8, F32)
        b["flat"] = torch.empty(B, 16 * d, device=self.dev, dtype=F32)
        b["u"] = torch.empty(B, self.flat.weight.shape[0], device=self.dev, dtype=F32)
        self._bufs[B] = b
        return b

    def _bn_fwd(self, B, key, mod, x, y, relu):
        st = self._bn_state(B, key, x.shape[0], x.shape[1])
        if mod.momentum is None:
            raise NotImplementedError("BatchNorm2d(momentum=None) (cumulative average) is not on the Encoder4 path")
        a = L.BatchNormArgs(rows=x.shape[0], c=x.shape[1], eps=mod.eps, momentum=mod.momentum, relu=int(relu),
                            x_f32=int(x.dtype == F32), x=x.data_ptr(), ldx=x.stride(0),
                            gamma=self.P(key + ".weight").data_ptr(),
                            beta=self.P(key + ".bias").data_ptr(), y=y.data_ptr(), ldy=y.stride(0),
                            y_split=int(y.shape[1] == 3 * x.shape[1]),
                            mean=st["mean"].data_ptr(), rstd=st["rstd"].data_ptr(),
                            running_mean=mod.running_mean.data_ptr() if mod.training else None,
                            running_var=mod.running_var.data_ptr() if mod.training else None,
                            partials=st["part"].data_ptr(), counter=st["counter"].data_ptr())
        L.check(L.lib.encdiff_batchnorm_fwd(C.byref(a), ops._s()), "encdiff_batchnorm_fwd")

    def _bn_bwd(self, B, key, mod, x, dy, dx, relu):
        st = self._bn_state(B, key, x.shape[0], x.shape[1])
        a = L.BatchNormArgs(rows=x.shape[0], c=x.shape[1], eps=mod.eps, momentum=mod.momentum, relu=int(relu),
                            x_f32=int(x.dtype == F32), x=x.data_ptr(), ldx=x.stride(0),
                            gamma=self.P(key + ".weight").data_ptr(),
                            beta=self.P(key + ".bias").data_ptr(), mean=st["mean"].data_ptr(),
                            rstd=st["rstd"].data_ptr(), partials=st["part"].data_ptr(),
                            counter=st["counter"].data_ptr(), dy=dy.data_ptr(), lddy=dy.stride(0),
                            dx=dx.data_ptr(), lddx=dx.stride(0), dgamma=self.G(key + ".weight").data_ptr(),
                            dbeta=self.G(key + ".bias").data_ptr())
        L.check(L.lib.encdiff_batchnorm_bwd(C.byref(a), ops._s()), "encdiff_batchnorm_bwd")

    def _bn_eval(self, B, key, mod, x, y, relu):
        """BatchNorm2d.eval() (+ReLU): the running statistics, no reduction."""
        st = self._bufs[B].get("bn_eval:" + key)
        if st is None:
            c = x.shape[1]
            st = self._bufs[B]["bn_eval:" + key] = dict(mean=torch.empty(c, device=self.dev),
                                                        rstd=torch.empty(c, device=self.dev))
        st["mean"].copy_(mod.running_mean)
        torch.rsqrt(mod.running_var + mod.eps, out=st["rstd"])
        a = L.BatchNormArgs(rows=x.shape[0], c=x.shape[1], eps=mod.eps, momentum=0.0, relu=int(relu),
                            x_f32=int(x.dtype == F32), x=x.data_ptr(), ldx=x.stride(0),
                            gamma=self.P(key + ".weight").data_ptr(), beta=self.P(key + ".bias").data_ptr(),
                            y=y.data_ptr(), ldy=y.stride(0), y_split=int(y.shape[1] == 3 * x.shape[1]),
                            mean=st["mean"].data_ptr(), rstd=st["rstd"].data_ptr())
        L.check(L.lib.encdiff_batchnorm_apply(C.byref(a), ops._s()), "encdiff_batchnorm_apply")

    # ------------------------------------------------------------ forward
    def forward(self, img: torch.Tensor, train: bool = True, head: bool = False) -> torch.Tensor:
        """img fp32 NCHW (B, 3, 64, 64) -> trunk output fp32 (B, d*16) in NCHW-flatten order, or
        with head=True the codes u = Linear(View(trunk)) (B, latent_unit) (encdiff_encoder_head_fwd on
        the NHWC rows: no flatten copy).  train=False: BatchNorm with the running statistics (eval
        mode; no backward)."""
        assert img.is_cuda and img.dtype == F32 and img.shape[1:] == (self.cin_img, self.img, self.img), \
            f"HIP Encoder4 trunk: fp32 (B, {self.cin_img}, {self.img}, {self.img}) device input"
        B = img.shape[0]
        b = self._bind(B)
        img = img.contiguous()
        d = self.d
        L.check(L.lib.encdiff_nchw_to_rows_split3(img.data_ptr(), B, self.cin_img, self.img * self.img, 8,
                                                  b["x0"].data_ptr(), 24,
                                                  ops._s()), "encdiff_nchw_to_rows_split3")
        bn = self._bn_fwd if train else self._bn_eval
        x = b["x0"]
        for i, c in enumerate(self.convs):
            g = Geom(B, c.hout, c.hout)
            w = self.pack.view("c0x3" if i == 0 else c.name + "x3")
            ops.conv4x4s2_fwd(x, g, x.shape[1], w, b[f"c{i}"], bias=self.P(c.name + ".bias"), out_f32=True)
            key, mod, relu = self.bns[i]
            y = b[f"a{i}"] if i < len(self.convs) - 1 else b["R0"][:, 3 * d:]  # the last one feeds res block 0
            bn(B, key, mod, b[f"c{i}"], y, relu)
            x = y
        g4 = Geom(B, 4, 4)
        for j, r in enumerate(self.res):
            p = r["prefix"]
            R = b[f"R{j}"]
            ops.conv3x3_fwd(R[:, 3 * d:], g4, 3 * d, self.pack.view(p + "1x3"), b[f"t{j}"], bias=self.P(p + "1.bias"),
                            out_f32=True)
            bn(B, p + "2", r["bn"], b[f"t{j}"], R[:, :3 * d], True)
            # r = h + conv1x1(u): [u_hi u_lo u_hi h_hi h_lo] x [W_hi W_hi W_lo I I]^T in one GEMM
            ops.linear_fwd(R[:, :5 * d], self.pack.view(p + "4x5"), b[f"r{j}"], bias=self.P(p + "4.bias"),
                           out_f32=True)
            if r["post_bn"] is not None:
                key, mod = r["post_bn"]
                bn(B, key, mod, b[f"r{j}"], b[f"R{j + 1}"][:, 3 * d:], True)
        if train and self.enc.training:
            self._count_batch()  # num_batches_tracked += 1 of every trunk BatchNorm2d (one launch)
        if head:
            r1, u = b["r1"], b["u"]
            L.check(L.lib.encdiff_encoder_head_fwd(r1.data_ptr(), r1.stride(0), B, d,
                                                   self.P(self.lin_name + ".weight").data_ptr(),
                                                   self.P(self.lin_name + ".bias").data_ptr(), u.shape[1],
                                                   u.data_ptr(), u.stride(0), ops._s()), "encdiff_encoder_head_fwd")
            return u
        flat = b["flat"]
        flat.view(B, d, 4, 4).copy_(b["r1"].view(B, 4, 4, d).permute(0, 3, 1, 2))
        return flat

    # ------------------------------------------------------------ backward
    def backward(self, d_flat: torch.Tensor, head: bool = False):
        """d_flat fp32 (B, d*16), NCHW-flatten order -> weight / BN gradients (+=) in the arena.
        head=True: d_flat is d u (B, latent_unit) of forward(head=True); the head's backward
        (encdiff_encoder_head_bwd) writes the trunk output gradient and the Linear's gradients."""
        B = d_flat.shape[0]
        b = self._bufs[B]
        d = self.d
        g4 = Geom(B, 4, 4)
        dh = b["dr1"]
        if head:
            du, r1 = d_flat.contiguous(), b["r1"]
            L.check(L.lib.encdiff_encoder_head_bwd(r1.data_ptr(), r1.stride(0), B, d,
                                                   self.P(self.lin_name + ".weight").data_ptr(), du.shape[1],
                                                   du.data_ptr(), du.stride(0), dh.data_ptr(), dh.stride(0),
                                                   self.G(self.lin_name + ".weight").data_ptr(),
                                                   self.G(self.lin_name + ".bias").data_ptr(), ops._s()),
                    "encdiff_encoder_head_bwd")
        else:
            dh.view(B, 4, 4, d).copy_(d_flat.view(B, d, 4, 4).permute(0, 2, 3, 1))
        for j in (1, 0):
            r = self.res[j]
            p = r["prefix"]
            R = b[f"R{j}"]
            if r["post_bn"] is not None:  # h_{j+1} = ReLU(BN(r_j))
                key, mod = r["post_bn"]
                self._bn_bwd(B, key, mod, b[f"r{j}"], dh, b[f"dr{j}"], True)
                dh = b[f"dr{j}"]
            # r = in + conv1x1(u): dgrad + wgrad of the 1x1 in one launch (u_hi = R[:, :d])
            ops.linear_bwd(dh, self.pack.view(p + "4"), R[:, :d], b[f"du{j}"],
                           self.G(p + "4.weight").view(d, d), self.G(p + "4.bias"))
            self._bn_bwd(B, p + "2", r["bn"], b[f"t{j}"], b[f"du{j}"], b[f"dt{j}"], True)
            # in-gradient = dh (residual) + conv3x3^T(dt): the residual rides the dgrad epilogue
            ops.conv3x3_bwd_cl(b[f"dt{j}"], g4, self.pack.view(p + "1"), R[:, 3 * d:4 * d], d,
                               self.Graw(p + "1.weight"), b[f"dh{j}"], self.G(p + "1.bias"), resid=dh)
            dh = b[f"dh{j}"]
        for i in range(len(self.convs) - 1, -1, -1):
            c = self.convs[i]
            key, mod, relu = self.bns[i]
            self._bn_bwd(B, key, mod, b[f"c{i}"], dh, b[f"dc{i}"], relu)
            dy = b[f"dc{i}"]
            g = Geom(B, c.hout, c.hout)
            if i == 0:  # the image has no gradient: weight gradient only (channel-padded, then folded)
                x = b["x0"]
                ops.gemm(c.cout, 16 * 8, g.pixels, dy, dy.stride(0), x, x.stride(0), b["dw0"], 16 * 8,
                         a_mode=L.OPA_ROWM, b_mode=L.OPB_IM2COL, c_mode=L.OUT_F32,
                         conv=L.ConvGeom(batch=B, h=c.hout, w=c.hout, cin=8, resample=L.RESAMPLE_K4S2,
                                         ld_src=x.stride(0)),
                         bias_grad=self.G(c.name + ".bias"))
                ops.flush()
                ops.grad_fold(b["dw0"], c.cout, self.cin_img, 8, 16, self.G(c.name + ".weight"))
                break
            x = b[f"a{i - 1}"][:, :d]  # the hi block of the split operand
            ops.conv4x4s2_bwd_cl(dy, g, self.pack.view(c.name), x, c.cin, self.Graw(c.name + ".weight"),
                                 b[f"da{i - 1}"], self.G(c.name + ".bias"))
            dh = b[f"da{i - 1}"]


class TrunkFn(torch.autograd.Function):
    """Encoder4 trunk + head on HIP: image -> codes u (B, latent_unit) fp32 (the trunk, View and
    Linear of Encoder4.encoder).  The parameters' gradients go straight to the arena (their .grad
    views); `anchor` (a trunk parameter) only makes the output require grad so the backward
    runs; the image gets no gradient."""

    @staticmethod
    def forward(ctx, img, anchor, ex):
        ctx.ex = ex
        return ex.forward(img, head=True)

    @staticmethod
    def backward(ctx, du):
        ctx.ex.backward(du, head=True)
        return None, None, None
