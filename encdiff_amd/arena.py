"""Flat parameter arena for the MI355X training step.

All trainable parameters of the denoiser (and, when training, of the concept
encoder) live in ONE fp32 buffer; each ``nn.Parameter`` keeps its reference name
and shape but its ``.data`` / ``.grad`` become views into the arena.  That makes

  * the optimizer one fused AdamW + EMA kernel over a contiguous array,
  * gradient all-reduce one (bucketable) contiguous buffer,
  * the per-step bf16 repack of GEMM weights one kernel driven by a job table.

The arena order is free (state_dict names are unaffected), so parameters that
the executor consumes together are laid out contiguously: the 28 ResBlock
emb_layers projections form one [sum 2C][256] matrix (one GEMM per step), the
16 cross-attention to_k/to_v projections one [sum 2C][context_dim] matrix, and
each self-attention's to_q/to_k/to_v one [3C][C] matrix.
"""
from __future__ import annotations

import os

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib as L


class ParamArena:
    """``channels_last``: names of [co][ci][kh][kw] conv weights stored as [co][kh][kw][ci]
    (the GEMM B layout, so the weight gradient is written coalesced and the bf16 pack is a
    plain cast); the parameter / grad / EMA views keep the reference shape through a
    permuted (strided) view."""

    def __init__(self, order: Sequence[Tuple[str, torch.nn.Parameter]], device, ema_names: Sequence[str] = (),
                 align: int = 8, channels_last: Sequence[str] = ()):
        self.device = torch.device(device)
        self.names: List[str] = []
        self.offsets: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
        self.params: Dict[str, torch.nn.Parameter] = {}
        self.cl = set(channels_last)
        off = 0
        ema_set = set(ema_names)
        # EMA-tracked params first so the EMA covers a prefix of the arena
        ordered = [o for o in order if o[0] in ema_set] + [o for o in order if o[0] not in ema_set]
        self.ema_numel = 0
        for name, p in ordered:
            if name in self.offsets:
                continue
            off = (off + align - 1) // align * align
            self.offsets[name] = (off, tuple(p.shape))
            self.params[name] = p
            self.names.append(name)
            off += p.numel()
            if name in ema_set:
                self.ema_numel = off
        self.numel = (off + 3) // 4 * 4
        self.master = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        self.grad = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        self.exp_avg = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        self.ema: Optional[torch.Tensor] = None
        with torch.no_grad():
            for name in self.names:
                p = self.params[name]
                view = self.view_in(self.master, name)
                view.copy_(p.detach().to(self.device, torch.float32))
                p.data = view
                p.grad = self.view_in(self.grad, name)
        self.step = 0
        self.hyper = torch.zeros(8, device=self.device, dtype=torch.float32)
        # bf16 shadow of the arena, index for index (enable_mirror): the GEMM operand copy of every
        # weight whose compute layout is its arena layout.  The fused optimizer writes it with the
        # update (encdiff_adamw_ema_mirror); mirror_fresh tells the packs it was just written.
        self.mirror: Optional[torch.Tensor] = None
        self.mirror_fresh = False
        # bumped by every host-side write of parameter values (EMA swap, load_state_dict):
        # consumers of bf16 weight copies (UNet / Encoder4 packs) repack when it moves.
        # Writes through a parameter's .data do not bump master._version (p.data is a view
        # with a version counter of its own), so this counter is the signal.
        self.gen = 0

    def mark_dirty(self):
        self.gen += 1

    # -------------------------------------------------------------- views
    def alias(self, local: str, name: str):
        """Address `name` also as `local` (e.g. UNet-local names inside a model arena)."""
        self.offsets[local] = self.offsets[name]
        if name in self.cl:
            self.cl.add(local)

    def view_in(self, base: torch.Tensor, name: str) -> torch.Tensor:
        """Reference-shaped view of `name` inside an arena-shaped buffer (master/grad/ema)."""
        o, shp = self.offsets[name]
        n = 1
        for s in shp:
            n *= s
        flat = base[o:o + n]
        if name in self.cl:
            co, ci, kh, kw = shp
            return flat.view(co, kh, kw, ci).permute(0, 3, 1, 2)
        return flat.view(shp)

    def raw(self, base: torch.Tensor, name: str) -> torch.Tensor:
        """Storage-order 2-D view [rows][cols] (conv weights: [co][kh*kw*ci])."""
        o, shp = self.offsets[name]
        n = 1
        for s in shp:
            n *= s
        return base[o:o + n].view(shp[0], n // shp[0])

    def f32(self, name: str) -> torch.Tensor:
        return self.view_in(self.master, name)

    def grad_of(self, name: str) -> torch.Tensor:
        return self.view_in(self.grad, name)

    def span(self, names: Sequence[str]) -> Tuple[int, int]:
        """(offset, numel) of a group of params laid out back-to-back (checked)."""
        o0, _ = self.offsets[names[0]]
        cur = o0
        for n in names:
            o, shp = self.offsets[n]
            assert o == cur, f"{n} not contiguous in the arena"
            k = 1
            for s in shp:
                k *= s
            cur = o + k
        return o0, cur - o0

    def attach_grads(self, zero: bool = True):
        """Make every parameter's .grad the arena view again (an optimizer's
        zero_grad(set_to_none=True) detaches them); re-attached slices start at zero (zero=False:
        the caller zeroes the whole arena itself, one launch instead of one per slice)."""
        for name in self.names:
            p = self.params[name]
            g = p.grad
            o, shp = self.offsets[name]
            if g is None or g.data_ptr() != self.grad.data_ptr() + 4 * o:
                view = self.view_in(self.grad, name)
                if zero:
                    view.zero_()
                p.grad = view

    def zero_grad(self):
        self.attach_grads(zero=False)
        self.grad.zero_()

    def enable_mirror(self) -> torch.Tensor:
        if self.mirror is None:
            self.mirror = self.master.to(torch.bfloat16)
        return self.mirror

    def enable_ema(self):
        if self.ema is None:
            self.ema = self.master[: self.ema_numel].clone()
        return self.ema


# plain-cast weights live in the arena's bf16 mirror, written by the optimizer with the update
# (0: every weight packed into the table's own buffer by encdiff_pack_weights, A/B runs)
MIRROR = os.environ.get("ENCDIFF_PACK_MIRROR", "1") != "0"


class PackTable:
    """bf16 compute copies of the GEMM weights.  Weights whose compute layout is their arena layout
    (kind 0: a plain cast) are views of the arena's bf16 mirror, which the fused optimizer writes
    with the update; the rest (permuted / padded / split-bf16 layouts) are packed from the fp32
    arena into this table's buffer by one kernel (encdiff_pack_weights) after every step."""

    def __init__(self, arena: ParamArena):
        self.arena = arena
        self.jobs: List[L.PackJob] = []
        self.mjobs: List[L.PackJob] = []  # mirror ranges (refreshed here only outside the optimizer)
        self.views: Dict[str, Tuple[int, int, int]] = {}  # key -> (dst_off, rows, cols)
        self.mviews: Dict[str, Tuple[int, int, int]] = {}  # key -> (arena offset, rows, cols)
        self.numel = 0

    def add(self, key: str, src_off: int, rows: int, cols: int, kind: int = 0, cin: int = 0):
        if MIRROR and kind == 0 and src_off % 8 == 0:
            self.mjobs.append(L.PackJob(src_off=src_off, dst_off=src_off, rows=rows, cols=cols, kind=0, cin=0))
            self.mviews[key] = (src_off, rows, cols)
            return
        off = (self.numel + 7) // 8 * 8
        self.jobs.append(L.PackJob(src_off=src_off, dst_off=off, rows=rows, cols=cols, kind=kind, cin=cin))
        # kind 6 (transpose): the copy is [cols][rows]
        self.views[key] = (off, cols, rows) if kind == 6 else (off, rows, cols)
        self.numel = off + rows * cols

    def finalize(self):
        dev = self.arena.device
        self.buf = torch.zeros(max(self.numel, 8), device=dev, dtype=torch.bfloat16)

        def table(jobs):
            arr = (L.PackJob * max(len(jobs), 1))(*jobs)
            return torch.frombuffer(bytearray(arr), dtype=torch.uint8).to(dev), len(jobs)
        self.jobs_dev, self.njobs = table(self.jobs)
        self.mjobs_dev, self.nmjobs = table(self.mjobs)
        if self.mjobs:
            self.arena.enable_mirror()

    def view(self, key: str) -> torch.Tensor:
        if key in self.mviews:
            off, rows, cols = self.mviews[key]
            return self.arena.mirror[off:off + rows * cols].view(rows, cols)
        off, rows, cols = self.views[key]
        return self.buf[off:off + rows * cols].view(rows, cols)

    def snapshot(self) -> torch.Tensor:
        """Every packed weight, concatenated (tests: did a repack happen)."""
        return torch.cat([self.buf] + [self.view(k).reshape(-1) for k in self.mviews])

    def repack(self):
        """Refresh every bf16 copy from the fp32 arena -- the mirror ranges too, unless the
        optimizer has just written them (arena.mirror_fresh)."""
        from . import ops
        if self.nmjobs and not self.arena.mirror_fresh:
            ops.pack_weights(self.arena.master, self.arena.mirror, self.mjobs_dev, self.nmjobs)
        if self.njobs:
            ops.pack_weights(self.arena.master, self.buf, self.jobs_dev, self.njobs)


class NormPartials:
    """Per-layer GroupNorm/LayerNorm gamma/beta partial sums laid out as columns of one
    fp32 matrix [rows][cols]; one encdiff_reduce_partials per step folds them into
    the gradient arena."""

    def __init__(self, arena: ParamArena, rows: int):
        self.arena = arena
        self.rows = rows
        self.cols = 0
        self.index: List[int] = []
        self.slots: Dict[str, int] = {}

    def add(self, gamma_name: str, beta_name: str) -> int:
        og, shg = self.arena.offsets[gamma_name]
        ob, shb = self.arena.offsets[beta_name]
        c = shg[0]
        base = self.cols
        self.index.extend(range(og, og + c))
        self.index.extend(range(ob, ob + c))
        self.cols += 2 * c
        self.slots[gamma_name] = base
        return base

    def finalize(self):
        dev = self.arena.device
        self.ld = max(self.cols, 1)
        self.buf = torch.zeros(self.rows, self.ld, device=dev, dtype=torch.float32)
        self.index_dev = torch.tensor(self.index if self.index else [0], device=dev, dtype=torch.int32)

    def parts(self, gamma_name: str, c: int):
        base = self.slots[gamma_name]
        return self.buf[:, base:base + c], self.buf[:, base + c:base + 2 * c]

    def reduce(self, lo: int = 0, hi: Optional[int] = None):
        """Fold columns [lo, hi) (default: all) into the gradient arena."""
        from . import ops
        hi = self.cols if hi is None else hi
        if hi > lo:
            ops.reduce_partials(self.buf[:, lo:], self.ld, self.rows, hi - lo, self.index_dev[lo:],
                                self.arena.grad)

    def split_col(self, sel) -> Optional[int]:
        """Column c such that the layers `sel(gamma_name)` selects own exactly [c, cols)
        (None when they do not form that suffix)."""
        names = sorted(self.slots, key=self.slots.get)
        flags = [bool(sel(n)) for n in names]
        if not any(flags):
            return self.cols
        k = flags.index(True)
        if not all(flags[k:]):
            return None
        return self.slots[names[k]]
