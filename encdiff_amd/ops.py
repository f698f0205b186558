"""Thin Python wrappers over the C-ABI (one call = one or two kernel launches).

Tensors are torch tensors used only as device memory; every call enqueues on
torch's current HIP stream, so the calls compose with torch ops and can be
captured into a HIP graph.  Activations are 2-D [rows][channels] bf16 views
(NHWC / token-major) whose row stride is passed as the leading dimension.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib as L
from ._lib import check, lib

BF16 = torch.bfloat16
F32 = torch.float32


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _ld(t: torch.Tensor) -> int:
    assert t.dim() == 2 and t.stride(1) == 1, "expected a row-major 2-D view"
    return t.stride(0)


@dataclass
class Geom:
    """Image geometry of an NHWC activation: `batch` images of h x w pixels."""
    batch: int
    h: int
    w: int

    @property
    def pixels(self):
        return self.batch * self.h * self.w


def _conv_geom(g: Geom, cin: int, resample: int, src: torch.Tensor) -> L.ConvGeom:
    return L.ConvGeom(batch=g.batch, h=g.h, w=g.w, cin=cin, resample=resample, ld_src=_ld(src))


_SCRATCH = {}
_RETIRED = []  # outgrown scratch stays allocated: graphs captured earlier still address it
# split-K GEMMs may combine their slabs in the kernel (EncdiffGemmArgs.split_counters) instead of
# a finalize launch: per problem, as the measured table says (4th entry).  ENCDIFF_SPLIT_FOLD:
# 1 table choice (default), 0 never, 2 always.
SPLIT_FOLD = int(os.environ.get("ENCDIFF_SPLIT_FOLD", "1"))
WS_FLOATS = 64 * 1024 * 1024         # fp32 split-K scratch per device, 256 MB (two halves, see gemm_pair)
WS_HALF = WS_FLOATS // 2
# the fused transformer blocks' grouped weight-gradient slabs (StWgrad): a scratch of their own, so
# a paired launch's deferred finalize (whose slabs sit in a split-K workspace half) can stay pending
# across a fused block's backward instead of being flushed as a launch of its own
STWG_WS_FLOATS = 24 * 1024 * 1024    # 96 MB (c = 64 / 128 at B = 128: 42 MB; larger batches: longer chunks)
COUNTERS = 1 << 16                   # split-K tickets per device (one int per output tile)
_TILES = None
_TILE_SHAPES = {1: (128, 128), 2: (128, 64), 3: (64, 128), 4: (64, 64)}


def scratch(name, numel, dtype=torch.float32, device=None):
    """Library scratch owned by this module, ONE per (device, name), allocated outside any graph
    capture and never freed.  Captured graphs hold these addresses, so they must not come from a
    graph's private memory pool (a pool dies with its graph; the old per-stream keying handed a
    dead graph's workspace to a later capture on a recycled stream handle).  Sharing one scratch
    per device is correct because every launch that uses it is ordered on one stream at a time:
    the executors issue GEMMs on the current stream only, and captured graphs are replayed one
    after another, never concurrently (the DP exchange stream runs collectives only)."""
    dev = torch.cuda.current_device() if device is None else device
    key = (dev, name)
    t = _SCRATCH.get(key)
    if t is None or t.numel() < numel:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"encdiff scratch '{name}' first needed inside a graph capture: run an eager "
                               f"step (or ops.ensure_scratch()) before capturing")
        if t is not None:
            _RETIRED.append(t)
        t = _SCRATCH[key] = torch.zeros(numel, device=f"cuda:{dev}", dtype=dtype)
    return t


def ensure_scratch(device=None):
    """Allocate the GEMM scratch now (executors call this at bind time, outside capture)."""
    _workspace(device)
    _counters(device)


def _counters(device=None):
    """Split-K tickets: one int per output tile, zero between launches (each launch's
    combining splits leave them zero)."""
    return scratch("split_counters", COUNTERS, torch.int32, device)


def _workspace(device=None):
    """Split-K slab scratch (fp32)."""
    return scratch("splitk_ws", WS_FLOATS, torch.float32, device)


def _tile_table():
    global _TILES
    if _TILES is None:
        import json
        import os
        path = os.environ.get("ENCDIFF_GEMM_TILES") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                    "gemm_tiles.json")
        _TILES = json.load(open(path)) if os.path.exists(path) else {}
    return _TILES


MAX_SPLIT = int(os.environ.get("ENCDIFF_MAX_SPLIT", "1024"))  # experiment knob: clamp table split-K
FORCE_TILE = 0  # tests: override the planned tile of every GEMM that does not pass one


# halo tiles (gemm.hip tiles 16-23): BM x BN, window staged once per workgroup
HALO_TILES = {16: (64, 64), 17: (128, 64), 18: (128, 128), 19: (256, 32), 20: (128, 32), 21: (256, 64),
              22: (64, 128), 23: (64, 32)}
HALO_LDS_MAX = 156 * 1024  # gemm.hip: 160 KiB less the paired kernel's static scratch


def halo_fits(tile, batch, h, w, cin, resample, split=1):
    """Host mirror of gemm.hip prepare_halo's geometry checks: the tile's BM pixels are whole
    rows of one image (or whole images) and window + 3-deep B ring + epilogue fit the LDS.
    split > 1: split-K by source-channel slices (cin / split channels per split, 64 | slice)."""
    if tile not in HALO_TILES or cin % 8 or resample not in (0, 2, 3, 4):
        return False
    if split > 1:
        if cin % (64 * split):
            return False
        cin //= split
    bm, bn = HALO_TILES[tile]
    hw = h * w
    if (batch * hw) % bm or bm % w or (hw % bm and bm % hw) or (resample == 2 and (h | w) & 1):
        return False
    s = 2 if resample in (3, 4) else 1
    kt = 4 if resample == 4 else 3
    rows = min(h, bm // w)
    ni = bm // hw if bm > hw else 1
    npix = ni * (s * (rows - 1) + kt) * (s * (w - 1) + kt)
    chunks = (npix * (cin // 8) + 255) & ~255
    return max(chunks * 16 + 3 * bn * 64 * 2, bm * (bn + 4) * 4) <= HALO_LDS_MAX


def plan_key(M, N, K, a_mode, b_mode, c_mode, resample=0, h=0):
    """Tile-table key.  h (the conv geometry's h, implicit-im2col problems): the same (M, N, K) is a
    different conv at another batch (B=512 at 8x8 has B=128 16x16's pixel count), and the halo
    and WG3 tiles are valid only for the geometry they were measured on -- keys written with h
    are looked up first, plain keys (older tables) after them."""
    key = f"{a_mode},{b_mode},{c_mode},{M},{N},{K}"
    return key + (f",r{resample}" if resample else "") + (f",h{h}" if h else "")


def _table_hit(M, N, K, a_mode, b_mode, c_mode, resample, h):
    t = _tile_table()
    for cm in ((c_mode, L.OUT_BF16) if c_mode == L.OUT_F32 else (c_mode,)):  # f32 output: the bf16 plan
        for hh in ((h, 0) if h else (0,)):
            hit = t.get(plan_key(M, N, K, a_mode, b_mode, cm, resample, hh))
            if hit is not None:
                return hit
    return None


def fold_choice(M, N, K, a_mode, b_mode, c_mode, resample=0, h=0) -> bool:
    """Whether a split-K GEMM combines its slabs in the kernel (measured per problem)."""
    if SPLIT_FOLD != 1:
        return SPLIT_FOLD == 2
    hit = _table_hit(M, N, K, a_mode, b_mode, c_mode, resample, h)
    return hit is not None and len(hit) > 3 and bool(hit[3])


def plan(M, N, K, a_mode, b_mode, c_mode, resample=0, h=0, table=True):
    """(tile, split_k) for a GEMM: measured table (tools/gemm_profile.py --write-table) first,
    else a heuristic aiming at >= 256 workgroups with bounded split-K traffic."""
    hit = _table_hit(M, N, K, a_mode, b_mode, c_mode, resample, h) if table else None
    if hit is not None:
        tile, split = int(hit[0]), min(int(hit[1]), MAX_SPLIT)
        if split == 1 or c_mode in (L.OUT_F32_ATOMIC, L.OUT_F32_ATOMIC_CONVW) or split * M * (N + 1) <= WS_FLOATS:
            return tile, split
    atomic = c_mode in (L.OUT_F32_ATOMIC, L.OUT_F32_ATOMIC_CONVW)
    bm = 64 if M <= 64 else 128
    bn = 64 if N <= 64 else 128

    def blocks(a, b):
        return math.ceil(M / a) * math.ceil(N / b)
    if blocks(bm, bn) < 512 and bm == 128:
        bm = 64
    if blocks(bm, bn) < 512 and bn == 128:
        bn = 64
    tile = {(128, 128): 1, (128, 64): 2, (64, 128): 3, (64, 64): 4}[(bm, bn)]
    nb = blocks(bm, bn)
    split = 1
    if atomic:
        while nb * split < 256 and K // (split * 2) >= 256 and (split * 2) * M * N * 4 <= (8 << 20):
            split *= 2
    else:  # slab split-K (bf16 / f32 / f32-accumulate outputs)
        while nb * split < 256 and K // (split * 2) >= 256 and (split * 2) * M * (N + 1) <= WS_HALF // 2:
            split *= 2
    return tile, split


WG3 = int(os.environ.get("ENCDIFF_WG3", "1"))  # 3x3 conv weight gradients on the WG3 kernel (tiles 32 / 33)
WG3_TILE = int(os.environ.get("ENCDIFF_WG3_TILE", "32"))  # 32: 3-deep stage ring, 33: 7-deep
WG3_SPLIT = 0  # experiments: force the WG3 split


def wg3_split(batch, h, w, cout, cin, resample, lda, ld_src, c_mode, tile=None):
    """Pixel chunks (split) of a 3x3 conv weight gradient on gemm.hip's WG3 kernel, or None when
    the problem is not eligible (mirror of gemm.hip wg3_check).  A workgroup owns 32 couts x 16
    cins x 9 taps of one chunk of whole images; its 4 (tile 32) or 8 (tile 33) waves split the
    chunk's 32-pixel stages: the largest power-of-two split whose waves still run >= 32 / waves
    stages and whose grid stays within 2 (4-wave) or 1 (8-wave) workgroups per CU, so the fp32
    partial slabs stay few."""
    tile = tile or WG3_TILE
    waves = 8 if tile == 33 else 4
    if (resample not in (L.RESAMPLE_NONE, L.RESAMPLE_UP2) or h != w or h not in (4, 8, 16) or cout % 32 or cin % 16
            or lda % 8 or ld_src % 8 or c_mode not in (L.OUT_F32, L.OUT_F32_ACCUM)):
        return None
    ni = 1 if h == 16 else 2
    rows = 4 if h == 4 else 2

    def stages(p):  # 32-pixel stages per chunk
        return (batch // p // ni) * (h // rows) if batch % (p * ni) == 0 else 0
    if not stages(1) or stages(1) % waves:
        return None
    nparts = (cout // 32) * (cin // 16)
    best, p = None, 1
    while stages(p) and stages(p) % waves == 0:
        if stages(p) // waves >= 32 // waves and nparts * p <= 256 * (2 if waves == 4 else 1):
            best = p
        p *= 2
    return best or 1


# tuned table entries for weight gradients over the WG3 / WGL heuristics (gemm_args): 0 off, 1 entries
# naming WG3 / WGL, 2 any entry
TABLE_WG = int(os.environ.get("ENCDIFF_TABLE_WG", "1"))

# linear weight gradients on the WGL kernel (tile 36): 0 off, 1 square c x c layers only, 2 every eligible one
WGL = int(os.environ.get("ENCDIFF_WGL", "1"))


def wgl_split(M, N, K, lda, ldb, c_mode):
    """Token chunks (split) of a linear weight gradient dW[M][N] += dY^T x on gemm.hip's WGL kernel
    (tile 36), or None when not eligible (mirror of gemm.hip wgl_check): workgroups own 64 x 64
    output parts, their 4 waves a quarter of a chunk each in 32-token stages; the largest
    power-of-two split whose waves still run >= 2 stages and whose grid stays <= 256 workgroups."""
    if M % 64 or N % 64 or lda % 8 or ldb % 8 or c_mode not in (L.OUT_F32, L.OUT_F32_ACCUM) or K % 256:
        return None
    parts = (M // 64) * (N // 64)
    best, p = None, 1
    while K % (p * 128) == 0:
        if K // (p * 128) >= 2 and parts * p <= 256:
            best = p
        p *= 2
    return best


def _plan_ok(tile, split, M, N, K, c_mode, conv, lda, ldb, a_mode=None) -> bool:
    """Whether a (tile, split) plan -- a table entry measured on some geometry -- is valid for THIS
    problem: halo tiles need the conv's window to fit (halo_fits), WG3 / WGL tiles their kernel's
    eligibility and a chunking that divides (wg3_check / wgl_check on the device side would raise
    ENCDIFF_ERR_SHAPE).  Keys carry (M, N, K, h) but not the batch, strides or alignment."""
    if tile in HALO_TILES:
        return (conv is not None and a_mode == L.OPA_IM2COL and
                halo_fits(tile, conv.batch, conv.h, conv.w, conv.cin, conv.resample, split))
    if tile in (32, 33, 34):
        if conv is None or wg3_split(conv.batch, conv.h, conv.w, M, conv.cin, conv.resample, lda, conv.ld_src,
                                     c_mode, tile=tile) is None:
            return False
        ni, rows = (1 if conv.h == 16 else 2), (4 if conv.h == 4 else 2)
        if conv.batch % (split * ni):
            return False
        return ((conv.batch // split // ni) * (conv.h // rows)) % (8 if tile == 33 else 4) == 0
    if tile == 36:
        return wgl_split(M, N, K, lda, ldb, c_mode) is not None and K % (split * 128) == 0
    return True


def gemm_args(M, N, K, a, lda, b, ldb, c, ldc, *, a_mode=L.OPA_ROWK, b_mode=L.OPB_ROWK, c_mode=L.OUT_BF16,
              conv: Optional[L.ConvGeom] = None, conv_cout=0, convw_cin=0, alpha=1.0, split_k=None, bias=None,
              resid=None, ld_resid=0, bias_grad=None, tile=0, ws_offset=0, aux=None, ld_aux=0,
              gn_stats=None, ln=None, agn=None, fold=False, plan_m=None, lna=None):
    """EncdiffGemmArgs with the measured (tile, split) plan; split-K slabs start `ws_offset`
    floats into this stream's workspace.  agn = (gamma, beta, film or None, eps, silu): GroupNorm of
    the im2col source applied in the A staging (tile 4); fold: split-K slabs combined in the kernel
    whenever the plan splits (the output is complete when the launch ends)."""
    if agn is not None:
        tile = 4
    if lna is not None:  # LayerNorm of the A rows in the staging: 64x64 tiles, no split
        tile, split_k = 4, 1
    if _WG_WHOLE:  # a WgradGroup member: whole problem, the group picks the body
        split_k = 1
    if TABLE_WG and tile == 0 and split_k is None and a_mode == L.OPA_ROWM:
        # a tuned table entry for this exact weight gradient (conv: keyed with its geometry) overrides
        # the WG3 / WGL split heuristics (1: entries naming those kernels, 2: any entry)
        im2 = conv is not None and b_mode == L.OPB_IM2COL
        hit = _tile_table().get(plan_key(M, N, K, a_mode, b_mode, c_mode, conv.resample if im2 else 0,
                                         conv.h if im2 else 0))
        if hit is not None and (TABLE_WG == 2 or int(hit[0]) in (32, 33, 34, 36)):
            t, sp = int(hit[0]), int(hit[1])
            if ((t not in (32, 33, 34) or WG3) and (t != 36 or WGL) and (sp == 1 or sp * M * (N + 1) <= WS_HALF // 2)
                    and _plan_ok(t, sp, M, N, K, c_mode, conv, lda, ldb, a_mode)):
                tile, split_k = t, sp
    if (WG3 and tile == 0 and split_k is None and a_mode == L.OPA_ROWM and b_mode == L.OPB_IM2COL and
            conv is not None and N == 9 * conv.cin and K == conv.batch * conv.h * conv.w):
        sp = wg3_split(conv.batch, conv.h, conv.w, M, conv.cin, conv.resample, lda, conv.ld_src, c_mode)
        if sp is not None and WG3_SPLIT:
            sp = WG3_SPLIT
        elif sp is not None and conv.batch == 128:  # measured pair split (tools/wg3_tune.py), training batch
            sp = _tile_table().get(f"wg3,{conv.h},{conv.cin},{M},{conv.resample}", sp)
        if sp is not None and (sp == 1 or sp * M * (N + 1) <= WS_HALF // 2):
            tile, split_k = WG3_TILE, sp
    if WGL and tile == 0 and split_k is None and a_mode == L.OPA_ROWM and b_mode == L.OPB_ROWN and (WGL == 2 or M == N):
        sp = wgl_split(M, N, K, lda, ldb, c_mode)
        if sp is not None and (sp == 1 or sp * M * (N + 1) <= WS_HALF // 2):
            tile, split_k = 36, sp
    pm = plan_m or M  # the row count whose measured plan is used (linear_fwd plan_m)
    rs = conv.resample if conv is not None else 0
    hk = conv.h if conv is not None and (a_mode == L.OPA_IM2COL or b_mode == L.OPB_IM2COL) else 0
    if split_k is None or tile == 0:
        t, sp = plan(pm, N, K, a_mode, b_mode, c_mode, rs, hk)
        if ((t in (32, 33, 34) and not WG3) or (t == 36 and not WGL) or  # kernel switched off, or a table
                not _plan_ok(t, sp, M, N, K, c_mode, conv, lda, ldb, a_mode)):  # plan invalid here: generic plan
            t, sp = plan(pm, N, K, a_mode, b_mode, c_mode, rs, hk, table=False)
        tile = tile or FORCE_TILE or t
        split_k = split_k or sp
    ws = None
    cnt = None
    if split_k > 1 and c_mode in (L.OUT_BF16, L.OUT_F32, L.OUT_F32_ACCUM):
        need = ws_offset + split_k * M * N + (split_k * M if bias_grad is not None else 0)
        assert need <= WS_FLOATS, "split-K slabs exceed the workspace"
        ws = _workspace()
        # the in-kernel combine indexes one ticket per output tile: only when every tile shape
        # (>= 32 x 32) stays within the ticket array
        if (a_mode != L.OPA_ROWM and math.ceil(M / 32) * math.ceil(N / 32) <= COUNTERS and
                (fold or fold_choice(pm, N, K, a_mode, b_mode, c_mode, rs, hk))):
            cnt = _counters()
    return L.GemmArgs(M=M, N=N, K=K, a_mode=a_mode, b_mode=b_mode, c_mode=c_mode,
                      a=_p(a), lda=lda, b=_p(b), ldb=ldb, c=_p(c), ldc=ldc,
                      conv=conv if conv is not None else L.ConvGeom(),
                      conv_cout=conv_cout, convw_cin=convw_cin, alpha=alpha, split_k=split_k,
                      bias=_p(bias), resid=_p(resid), ld_resid=ld_resid, bias_grad=_p(bias_grad), tile=tile,
                      workspace=None if ws is None else ws.data_ptr() + 4 * ws_offset, aux=_p(aux), ld_aux=ld_aux,
                      gn_stats=_p(gn_stats), ld_gn_stats=_ld(gn_stats) if gn_stats is not None else 0,
                      split_counters=None if cnt is None else cnt.data_ptr(),
                      **({} if ln is None else dict(ln_gamma=_p(ln[0]), ln_beta=_p(ln[1]), ln_y=_p(ln[2]),
                                                    ld_ln_y=_ld(ln[2]), ln_stats=_p(ln[3]), ln_eps=ln[4])),
                      **({} if agn is None else dict(agn_gamma=_p(agn[0]), agn_beta=_p(agn[1]), agn_film=_p(agn[2]),
                                                     ld_agn_film=_ld(agn[2]) if agn[2] is not None else 0,
                                                     agn_eps=agn[3], agn_silu=int(agn[4]))),
                      **({} if lna is None else dict(lna_gamma=_p(lna[0]), lna_beta=_p(lna[1]), lna_eps=lna[2])))


def ws_floats(args) -> int:
    """Workspace floats a GEMM's split-K slabs (+ bias-gradient slabs) occupy, rounded up to
    16 bytes so a slab region placed behind it keeps the finalize's float4 loads aligned."""
    if args.split_k <= 1 or args.c_mode not in (L.OUT_BF16, L.OUT_F32, L.OUT_F32_ACCUM):
        return 0
    n = args.split_k * args.M * args.N + (args.split_k * args.M if args.bias_grad else 0)
    return (n + 3) & ~3


# Keyed by DEVICE, like the workspace the slabs live in (scratch()): a finalize left pending by a
# launch on one stream is flushed by the next workspace user on any stream of that device.
_PENDING = {}  # device -> (GemmArgs, producing stream) of a weight gradient whose split-K finalize is deferred
_HALF = {}     # device -> workspace half used by the last paired launch


def _take_pending(key):
    """The deferred weight-gradient finalize of this device, ordered after its producer: when the
    GEMM that left it ran on another stream, the current stream waits for that stream first (the
    finalize reads its slabs)."""
    ent = _PENDING.pop(key, None)
    if ent is None:
        return None
    args, producer = ent
    cur = torch.cuda.current_stream()
    if producer != cur:
        cur.wait_stream(producer)
    return args


def flush():
    """Run the deferred weight-gradient finalize of this device, if any (the end of a backward, or
    before a GEMM that needs the workspace)."""
    pend = _take_pending(torch.cuda.current_device())
    if pend is not None:
        check(lib.encdiff_gemm_finalize(C.byref(pend), _s()), "encdiff_gemm_finalize")


def gemm(M, N, K, a, lda, b, ldb, c, ldc, **kw):
    args = gemm_args(M, N, K, a, lda, b, ldb, c, ldc, **kw)
    if ws_floats(args):
        flush()  # its slabs start at offset 0: the deferred slabs must be consumed first
    check(lib.encdiff_gemm(C.byref(args), _s()), "encdiff_gemm")


PAIR = True  # fuse a layer's weight- and input-gradient GEMMs into one launch (encdiff_gemm_pair_ex)

# Grouped weight gradients (encdiff_wgrad_group_*): while a WgradGroup is active, gemm_pair and
# linear_wgrad launch only the input gradient and hand the weight gradient (whole: split_k 1) to
# the group, which runs all of them as ONE grid at group_end().  ENCDIFF_WG_GROUP=0: paired launches.
WG_GROUP = int(os.environ.get("ENCDIFF_WG_GROUP", "0"))  # measured slower than the pairs: DESIGN.md §5
# only weight gradients with K (pixels / tokens) <= WG_MAXK join the group; deeper ones stay paired
# with their input gradient (their grid overlaps the input gradient's latency-bound tiles)
WG_MAXK = int(os.environ.get("ENCDIFF_WG_MAXK", str(1 << 30)))
_GROUP = None      # the active WgradGroup
_WG_WHOLE = False  # gemm_args: build a weight gradient for the group (split_k 1, no slabs)


GROUP_PROBS = {}  # host blob address of a planned group -> its problems (bench.py's GEMM-family record)


class WgradGroup:
    """The weight-gradient GEMMs of a backward region, launched together.  Launch descriptions
    are planned once per distinct problem list (the executors' buffers are static per batch size,
    so a list recurs bit for bit every step) and kept in device memory for the life of the group:
    captured graphs read them at replay."""

    def __init__(self):
        self.probs = []
        self._plans = {}

    def add(self, args):
        self.probs.append(args)

    def launch(self):
        probs, self.probs = self.probs, []
        if not probs:
            return
        arr = (L.GemmArgs * len(probs))(*probs)
        key = bytes(arr)
        ent = self._plans.get(key)
        if ent is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("encdiff weight-gradient group first planned inside a graph capture: run an "
                                   "eager step before capturing")
            # chunk slabs in the workspace's second half (the first holds deferred input-gradient
            # slabs until their norms consume them -- all before the group runs)
            sc = (_workspace().data_ptr() + 4 * WS_HALF, WS_HALF, _counters().data_ptr(), COUNTERS)
            nb = C.c_long(0)
            check(lib.encdiff_wgrad_group_plan(arr, len(probs), *sc, None, 0, C.byref(nb)), "encdiff_wgrad_group_plan")
            host = (C.c_longlong * ((nb.value + 7) // 8))()
            check(lib.encdiff_wgrad_group_plan(arr, len(probs), *sc, C.addressof(host), C.sizeof(host), C.byref(nb)),
                  "encdiff_wgrad_group_plan")
            dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(torch.cuda.current_device())
            ent = self._plans[key] = (host, dev, probs)  # (the problems: tools / tests re-plan subsets)
            GROUP_PROBS[C.addressof(host)] = probs
        check(lib.encdiff_wgrad_group_launch(C.addressof(ent[0]), ent[1].data_ptr(), _s()), "encdiff_wgrad_group_launch")


def group_begin(group: Optional[WgradGroup]):
    """Route the following weight gradients into `group` (None: launch them as before)."""
    global _GROUP
    _GROUP = group


def group_flush():
    """Launch the weight gradients collected so far; the group stays active (windowed groups: the
    dY / x operands of the last few blocks are still resident in the 256 MB Infinity Cache)."""
    if _GROUP is not None:
        flush()  # a paired launch's deferred finalize: its slabs share the group's workspace half
        _GROUP.launch()


def group_end():
    """Launch the active group's weight gradients and deactivate it."""
    global _GROUP
    g, _GROUP = _GROUP, None
    if g is not None:
        flush()
        g.launch()


def _grouped(wgrad_fn):
    """The whole-problem weight gradient of `wgrad_fn` added to the active group, or None when
    no group is active or the problem is deeper than WG_MAXK (it runs paired / alone)."""
    if _GROUP is None:
        return None
    w = _whole_wgrad(wgrad_fn)
    if w.K > WG_MAXK:
        return None
    _GROUP.add(w)
    return w


def _whole_wgrad(wgrad_fn):
    global _WG_WHOLE
    _WG_WHOLE = True
    try:
        return wgrad_fn(0)
    finally:
        _WG_WHOLE = False


def _dgrad_alone(d, defer_dx):
    if ws_floats(d):
        flush()
    if not defer_dx:
        check(lib.encdiff_gemm(C.byref(d), _s()), "encdiff_gemm")
        return None
    planned = C.c_int(0)
    check(lib.encdiff_gemm_ex(C.byref(d), 1, C.byref(planned), _s()), "encdiff_gemm_ex")
    return d if planned.value else None


def gemm_pair(wgrad_fn, dgrad_fn, defer_dx=False):
    """Launch a layer's weight-gradient and input-gradient GEMMs together (`wgrad_fn(off)`,
    `dgrad_fn(off)` build their GemmArgs with split-K slabs at workspace offset `off`).
    Consecutive pairs alternate between the two workspace halves: the weight gradient's
    finalize is deferred into the NEXT pair's launch (its slabs stay intact in the other
    half), so a backward of N layers needs no finalize launches for weight gradients but the
    last (`flush`).  defer_dx: the input gradient's finalize is skipped too when it has one;
    its GemmArgs are returned for the consumer (groupnorm_bwd(dy_from=...)) or finalize(),
    which must run before the next pair (else None: dx written).
    With a WgradGroup active the weight gradient goes to the group and only the input gradient
    is launched here."""
    if _grouped(wgrad_fn) is not None:
        return _dgrad_alone(dgrad_fn(0), defer_dx)
    key = torch.cuda.current_device()
    if not PAIR:
        flush()
        w = wgrad_fn(0)
        d = dgrad_fn(ws_floats(w))
        check(lib.encdiff_gemm(C.byref(w), _s()), "encdiff_gemm")
        check(lib.encdiff_gemm(C.byref(d), _s()), "encdiff_gemm")
        return None
    w = wgrad_fn(0)
    nw = ws_floats(w)
    if nw + ws_floats(dgrad_fn(0)) > WS_HALF:  # does not fit a half: plain pair, whole workspace
        flush()
        d = dgrad_fn(nw)
        check(lib.encdiff_gemm_pair(C.byref(w), C.byref(d), _s()), "encdiff_gemm_pair")
        return None
    h = 1 - _HALF.get(key, 1)
    if h:
        w = wgrad_fn(h * WS_HALF)
    d = dgrad_fn(h * WS_HALF + nw)
    prev = _take_pending(key)
    dd = C.c_int(0)
    check(lib.encdiff_gemm_pair_dx(C.byref(w), C.byref(d), C.byref(prev) if prev is not None else None, 1,
                                   int(defer_dx), C.byref(dd), _s()), "encdiff_gemm_pair_dx")
    if nw:
        _PENDING[key] = (w, torch.cuda.current_stream())
    _HALF[key] = h
    return d if dd.value else None


# ------------------------------------------------------------------ linear layers
def linear_fwd(x, w, out, bias=None, resid=None, alpha=1.0, out_f32=False, gn_stats=None, plan_m=None,
               ln_in=None):
    """out[M][N] = x[M][K] w[N][K]^T (+bias)(+resid); gn_stats: [2*M/64][ld] fp32 view that
    receives the per-64-row-segment channel sums of out (the next GroupNorm's statistics).
    plan_m: take the (tile, split, fold) plan of the same problem with plan_m rows, so every row
    comes out bitwise as that smaller GEMM computes it (the sampler's per-loop FiLM table).
    ln_in = (gamma, beta, eps): out = LayerNorm(x) w^T (+bias)(+resid), the LayerNorm applied to
    the staged A tiles (EncdiffGemmArgs.lna_*; inference: no normalised rows materialised)."""
    M, K = x.shape
    N = w.shape[0]
    gemm(M, N, K, x, _ld(x), w, _ld(w), out, _ld(out), c_mode=L.OUT_F32 if out_f32 else L.OUT_BF16,
         bias=bias, resid=resid, ld_resid=_ld(resid) if resid is not None else 0, alpha=alpha,
         gn_stats=gn_stats, split_k=1 if gn_stats is not None else None, plan_m=plan_m, lna=ln_in)


# LayerNorm in the producing GEMM's epilogue when one tile spans the row (N <= 128):
# attention.py norm1/2/3 after proj_in / to_out.  ENCDIFF_LN_FUSED=0: separate kernel.
LN_FUSED = os.environ.get("ENCDIFF_LN_FUSED", "1") != "0"
_TILE_BN = {1: 128, 2: 64, 3: 128, 4: 64, 5: 64, 6: 128, 7: 64, 8: 128}


def linear_fwd_ln(x, w, out, gamma, beta, y, stats, eps, bias=None, resid=None):
    """out = x w^T (+bias)(+resid), then y = LayerNorm(out) with per-row (mean, rstd) stats; in
    the GEMM epilogue when the planned tile spans the row, else the LayerNorm kernel."""
    M, K = x.shape
    N = w.shape[0]
    if not LN_FUSED or N > 128 or N % 8:
        linear_fwd(x, w, out, bias=bias, resid=resid)
        layernorm_fwd(out, gamma, beta, y, stats, eps)
        return
    tile, _ = plan(M, N, K, L.OPA_ROWK, L.OPB_ROWK, L.OUT_BF16)
    if M < 8192:
        # small (sampling) batches: a launch saved outweighs the tile choice -- force a tile that
        # spans the row (split-K 1; these GEMMs have K = C <= 512, a few k-tiles)
        if K > 512:
            linear_fwd(x, w, out, bias=bias, resid=resid)
            layernorm_fwd(out, gamma, beta, y, stats, eps)
            return
        tile = 3 if N > 64 else 4
    elif _TILE_BN.get(tile, 64) < N:  # at training batch sizes forcing a wider tile measured slower
        linear_fwd(x, w, out, bias=bias, resid=resid)
        layernorm_fwd(out, gamma, beta, y, stats, eps)
        return
    gemm(M, N, K, x, _ld(x), w, _ld(w), out, _ld(out), bias=bias, resid=resid,
         ld_resid=_ld(resid) if resid is not None else 0, split_k=1, tile=tile,
         ln=(gamma, beta, y, stats.view(-1, 2) if stats.dim() != 2 else stats, eps))


def linear_dgrad(dy, w, dx, resid=None):
    """dx[M][K] = dy[M][N] w[N][K] (+resid, e.g. dx itself to accumulate)."""
    M, N = dy.shape
    K = w.shape[1]
    gemm(M, K, N, dy, _ld(dy), w, _ld(w), dx, _ld(dx), b_mode=L.OPB_ROWN,
         resid=resid, ld_resid=_ld(resid) if resid is not None else 0)


def linear_dgrad_args(dy, w, dx, resid=None, ws_offset=0):
    M, N = dy.shape
    K = w.shape[1]
    return gemm_args(M, K, N, dy, _ld(dy), w, _ld(w), dx, _ld(dx), b_mode=L.OPB_ROWN,
                     resid=resid, ld_resid=_ld(resid) if resid is not None else 0, ws_offset=ws_offset)


def linear_wgrad_args(dy, x, dw, db=None, ws_offset=0):
    M, N = dy.shape
    K = x.shape[1]
    return gemm_args(N, K, M, dy, _ld(dy), x, _ld(x), dw, K, a_mode=L.OPA_ROWM, b_mode=L.OPB_ROWN,
                     c_mode=L.OUT_F32_ACCUM, bias_grad=db, ws_offset=ws_offset)


def linear_wgrad(dy, x, dw, db=None):
    """dw[N][K] += dy[M][N]^T x[M][K] (split-K slabs summed in order: reproducible);
    db[N] += sum_m dy[m][n]."""
    if _grouped(lambda off: linear_wgrad_args(dy, x, dw, db, off)) is not None:
        return
    args = linear_wgrad_args(dy, x, dw, db)
    if ws_floats(args):
        flush()
    check(lib.encdiff_gemm(C.byref(args), _s()), "encdiff_gemm")


def linear_bwd(dy, w, x, dx, dw, db=None, resid=None, defer_dx=False):
    """Backward of one linear layer: dw += dy^T x (+ db), dx = dy w (+ resid), one launch
    (defer_dx: as gemm_pair)."""
    return gemm_pair(lambda off: linear_wgrad_args(dy, x, dw, db, off),
                     lambda off: linear_dgrad_args(dy, w, dx, resid, off), defer_dx=defer_dx)


# GEGLU feed-forward (attention.py GEGLU / FeedForward): the activation runs in the GEMM
# epilogues -- the proj GEMM writes f and y = f_value * gelu(f_gate); the next layer's input
# gradient GEMM turns its dy tile into df.  ENCDIFF_GEGLU_FUSED=0: separate ew launches.
GEGLU_FUSED = os.environ.get("ENCDIFF_GEGLU_FUSED", "1") != "0"


def linear_fwd_geglu(x, w, f, y, bias=None):
    """f[M][2I] = x w^T (+bias); y[M][I] = f[:, :I] * gelu(f[:, I:])."""
    M, K = x.shape
    N = w.shape[0]
    if not GEGLU_FUSED or N % 128:
        linear_fwd(x, w, f, bias=bias)
        geglu_fwd(f, y)
        return
    gemm(M, N, K, x, _ld(x), w, _ld(w), f, _ld(f), c_mode=L.OUT_BF16_GEGLU, bias=bias, split_k=1, aux=y,
         ld_aux=_ld(y))


def linear_bwd_geglu(dy, w, a, f, df, dw, db=None, d_a=None):
    """Backward of y2 = Linear(GEGLU(f)): dw += dy^T a (+ db) and df = GEGLU'(f) * (dy w), the
    GEGLU backward in the input-gradient GEMM's epilogue (d_a: scratch of the unfused path)."""
    if not GEGLU_FUSED or 2 * w.shape[1] % 128:
        linear_bwd(dy, w, a, d_a, dw, db)
        geglu_bwd(f, d_a, df)
        return
    M = dy.shape[0]
    inner = w.shape[1]

    def dargs(off):
        return gemm_args(M, inner, w.shape[0], dy, _ld(dy), w, _ld(w), df, _ld(df), b_mode=L.OPB_ROWN,
                         c_mode=L.OUT_BF16_GEGLU_BWD, split_k=1, aux=f, ld_aux=_ld(f), ws_offset=off)
    gemm_pair(lambda off: linear_wgrad_args(dy, a, dw, db, off), dargs)


# ------------------------------------------------------------------ 3x3 convolutions
def conv3x3_fwd(x, g: Geom, cin, wf, out, bias=None, resid=None, resample=L.RESAMPLE_NONE, gn_stats=None,
                out_f32=False, defer=False, agn=None, fold=False):
    """out[pixels][cout] = conv3x3(resample(x)) with packed weights wf [cout][9*cin]
    (gn_stats: as linear_fwd; out_f32: fp32 output).  defer: when the plan leaves split-K slabs
    for a finalize pass, skip it and return the GemmArgs -- the caller hands them to
    groupnorm_fwd(x_from=...) (which writes `out`) or to finalize(); else None (out written).
    agn = (gamma, beta, film or None, eps, silu): the conv reads GroupNorm(+FiLM)(+SiLU)(x) -- applied
    in its A staging, x complete -- instead of a GroupNorm output; fold: see gemm_args."""
    cout = wf.shape[0]
    args = gemm_args(g.pixels, cout, 9 * cin, x, _ld(x), wf, _ld(wf), out, _ld(out), a_mode=L.OPA_IM2COL,
                     c_mode=L.OUT_F32 if out_f32 else L.OUT_BF16, conv=_conv_geom(g, cin, resample, x), bias=bias,
                     resid=resid, ld_resid=_ld(resid) if resid is not None else 0, gn_stats=gn_stats,
                     split_k=1 if gn_stats is not None else None, agn=agn, fold=fold)
    if ws_floats(args):
        flush()
    if not defer:
        check(lib.encdiff_gemm(C.byref(args), _s()), "encdiff_gemm")
        return None
    planned = C.c_int(0)
    check(lib.encdiff_gemm_ex(C.byref(args), 1, C.byref(planned), _s()), "encdiff_gemm_ex")
    return args if planned.value else None


def finalize(args):
    """Run the split-K finalize a deferred conv3x3_fwd left (no-op for None)."""
    if args is not None:
        check(lib.encdiff_gemm_finalize(C.byref(args), _s()), "encdiff_gemm_finalize")


def conv3x3_dgrad(dy, g: Geom, wf, dx, resid=None):
    """dx[pixels][cin] = conv3x3^T(dy) (input grad at the conv resolution)."""
    cout = wf.shape[0]
    cin = wf.shape[1] // 9
    gemm(g.pixels, cin, 9 * cout, dy, _ld(dy), wf, _ld(wf), dx, _ld(dx), a_mode=L.OPA_IM2COL,
         b_mode=L.OPB_CONV_DGRAD, conv=_conv_geom(g, cout, L.RESAMPLE_NONE, dy), conv_cout=cout,
         resid=resid, ld_resid=_ld(resid) if resid is not None else 0)


def conv3x3_wgrad(dy, x, g: Geom, cin, dw_ref, db=None, resample=L.RESAMPLE_NONE):
    """dw_ref[cout][cin][3][3] (fp32, reference layout) += sum_pix dy^T im2col(resample(x))."""
    cout = dy.shape[1]
    M, N, K = cout, 9 * cin, g.pixels
    gemm(M, N, K, dy, _ld(dy), x, _ld(x), dw_ref, 9 * cin, a_mode=L.OPA_ROWM, b_mode=L.OPB_IM2COL,
         c_mode=L.OUT_F32_ATOMIC_CONVW, conv=_conv_geom(g, cin, resample, x), convw_cin=cin, bias_grad=db)


def conv3x3_wgrad_cl_args(dy, x, g: Geom, cin, dw_cl, db=None, resample=L.RESAMPLE_NONE, ws_offset=0):
    cout = dy.shape[1]
    return gemm_args(cout, 9 * cin, g.pixels, dy, _ld(dy), x, _ld(x), dw_cl, _ld(dw_cl), a_mode=L.OPA_ROWM,
                     b_mode=L.OPB_IM2COL, c_mode=L.OUT_F32_ACCUM, conv=_conv_geom(g, cin, resample, x),
                     bias_grad=db, ws_offset=ws_offset)


def conv3x3_wgrad_cl(dy, x, g: Geom, cin, dw_cl, db=None, resample=L.RESAMPLE_NONE):
    """dw_cl[cout][9*cin] (fp32, channels-last [co][kh][kw][ci]) += dy^T im2col(resample(x))
    (split-K slabs summed in order: reproducible)."""
    if _grouped(lambda off: conv3x3_wgrad_cl_args(dy, x, g, cin, dw_cl, db, resample, off)) is not None:
        return
    args = conv3x3_wgrad_cl_args(dy, x, g, cin, dw_cl, db, resample)
    if ws_floats(args):
        flush()
    check(lib.encdiff_gemm(C.byref(args), _s()), "encdiff_gemm")


def conv3x3_dgrad_args(dy, g: Geom, wf, dx, resid=None, ws_offset=0):
    cout = wf.shape[0]
    cin = wf.shape[1] // 9
    return gemm_args(g.pixels, cin, 9 * cout, dy, _ld(dy), wf, _ld(wf), dx, _ld(dx), a_mode=L.OPA_IM2COL,
                     b_mode=L.OPB_CONV_DGRAD, conv=_conv_geom(g, cout, L.RESAMPLE_NONE, dy), conv_cout=cout,
                     resid=resid, ld_resid=_ld(resid) if resid is not None else 0, ws_offset=ws_offset)


def conv3x3_bwd_cl(dy, g: Geom, wf, x, cin, dw_cl, dx, db=None, resample=L.RESAMPLE_NONE, resid=None,
                   defer_dx=False):
    """Backward of one 3x3 conv: dw_cl += dy^T im2col(resample(x)) (+ db) and
    dx = conv3x3^T(dy) (+ resid) at the conv resolution, one launch (defer_dx: as gemm_pair)."""
    return gemm_pair(lambda off: conv3x3_wgrad_cl_args(dy, x, g, cin, dw_cl, db, resample, off),
                     lambda off: conv3x3_dgrad_args(dy, g, wf, dx, resid, off), defer_dx=defer_dx)


# ------------------------------------------------------------------ 4x4 stride-2 convolutions
def conv4x4s2_fwd(x, g_out: Geom, cin, wf, out, bias=None, out_f32=False):
    """Conv2d(k4, s2, p1) (Encoder4, openaimodel_enc.py:1002-1009): x at (2h, 2w), out at
    g_out = (h, w); wf packed [cout][16*cin] ([co][kh][kw][ci]); out_f32: fp32 output."""
    cout = wf.shape[0]
    gemm(g_out.pixels, cout, 16 * cin, x, _ld(x), wf, _ld(wf), out, _ld(out), a_mode=L.OPA_IM2COL,
         c_mode=L.OUT_F32 if out_f32 else L.OUT_BF16,
         conv=L.ConvGeom(batch=g_out.batch, h=g_out.h, w=g_out.w, cin=cin, resample=L.RESAMPLE_K4S2,
                         ld_src=_ld(x)), bias=bias)


K4S2_PARITY = True  # tests: False forces the 16-tap K4S2_T input gradient


def conv4x4s2_bwd_cl(dy, g_out: Geom, wf, x, cin, dw_cl, dx, db=None):
    """Backward of Conv2d(k4, s2, p1): dw_cl[cout][16*cin] += dy^T im2col(x) (+ db) and
    dx (2h, 2w) = transposed conv of dy, one paired launch."""
    cout = wf.shape[0]
    gin = Geom(g_out.batch, 2 * g_out.h, 2 * g_out.w)
    def wargs(off):
        return gemm_args(cout, 16 * cin, g_out.pixels, dy, _ld(dy), x, _ld(x), dw_cl, _ld(dw_cl),
                         a_mode=L.OPA_ROWM, b_mode=L.OPB_IM2COL, c_mode=L.OUT_F32_ACCUM,
                         conv=L.ConvGeom(batch=g_out.batch, h=g_out.h, w=g_out.w, cin=cin,
                                         resample=L.RESAMPLE_K4S2, ld_src=_ld(x)), bias_grad=db, ws_offset=off)

    # by output parity (2x2 taps each, K = 4*cout) when a GEMM tile never straddles two
    # parity classes, else all 16 taps with 3 of 4 masked
    tp = K4S2_PARITY and (gin.pixels // 4) % 128 == 0

    def dargs(off):
        return gemm_args(gin.pixels, cin, (4 if tp else 16) * cout, dy, _ld(dy), wf, _ld(wf), dx, _ld(dx),
                         a_mode=L.OPA_IM2COL, b_mode=L.OPB_CONV_DGRAD,
                         conv=L.ConvGeom(batch=gin.batch, h=gin.h, w=gin.w, cin=cout,
                                         resample=L.RESAMPLE_K4S2_TP if tp else L.RESAMPLE_K4S2_T, ld_src=_ld(dy)),
                         conv_cout=cout, ws_offset=off)
    gemm_pair(wargs, dargs)


# ------------------------------------------------------------------ normalisation
def groupnorm_fwd(x, g: Geom, gamma, beta, y, stats, eps, silu, film=None, ld_film=0, groups=32, in_stats=None,
                  x_from=None, dsilu=None):
    """in_stats: the segment sums x's producer GEMM wrote (gn_stats), else a reduction pass.
    x_from: the GemmArgs a deferred conv3x3_fwd returned for x -- its slabs are combined here
    (x written, bitwise the finalize's result), one launch instead of two.  dsilu (training, with
    silu): bf16 rows [pixels][c] that receive silu'(z) for the backward (groupnorm_bwd(dsilu=))."""
    c = x.shape[1]
    a = L.GroupNormArgs(batch=g.batch, hw=g.h * g.w, c=c, groups=groups, eps=eps, silu=int(silu),
                        x=_p(x), ldx=_ld(x), gamma=_p(gamma), beta=_p(beta), film=_p(film), ld_film=ld_film,
                        y=_p(y), ldy=_ld(y), stats=_p(stats), in_stats=_p(in_stats),
                        ld_in_stats=_ld(in_stats) if in_stats is not None else 0,
                        x_from=None if x_from is None else C.addressof(x_from),
                        dsilu=_p(dsilu), ld_dsilu=_ld(dsilu) if dsilu is not None else 0)
    check(lib.encdiff_groupnorm_fwd(C.byref(a), _s()), "encdiff_groupnorm_fwd")


def groupnorm_bwd(x, g: Geom, gamma, beta, stats, eps, silu, dy, dx, dgamma_part, dbeta_part, film=None,
                  ld_film=0, dfilm=None, ld_dfilm=0, accumulate=False, groups=32, ld_part=None, resid=None,
                  dy_from=None, dy_resample=0, resid_resample=0, dsilu=None, fold=None):
    """dx (+)= GN_bwd(dy) (+ resid: the block's skip-branch gradient, added in the same pass).
    dsilu: the forward's silu'(z) rows (groupnorm_fwd(dsilu=)), read instead of recomputed.
    fold: (device plan, blocks) of StWgrad.launch(..., ride=True): that plan's chunk fold runs as
    extra workgroups of this launch.
    dy_from: the GemmArgs of dy's producer whose finalize gemm_pair deferred (dy written here).
    dy_resample / resid_resample: dy / resid are at the resolution of that 2x resample following
    the GroupNorm (L.RESAMPLE_DOWN2 / UP2); their adjoint is applied on the fly."""
    c = x.shape[1]
    a = L.GroupNormArgs(batch=g.batch, hw=g.h * g.w, c=c, groups=groups, eps=eps, silu=int(silu),
                        x=_p(x), ldx=_ld(x), gamma=_p(gamma), beta=_p(beta), film=_p(film), ld_film=ld_film,
                        stats=_p(stats), dy=_p(dy), lddy=_ld(dy), dx=_p(dx), lddx=_ld(dx),
                        accumulate_dx=int(accumulate), dgamma_part=_p(dgamma_part), dbeta_part=_p(dbeta_part),
                        ld_part=c if ld_part is None else ld_part, dfilm=_p(dfilm), ld_dfilm=ld_dfilm,
                        resid=_p(resid), ld_resid=_ld(resid) if resid is not None else 0,
                        x_from=None if dy_from is None else C.addressof(dy_from), dy_resample=dy_resample,
                        resid_resample=resid_resample, w=g.w,
                        dsilu=_p(dsilu), ld_dsilu=_ld(dsilu) if dsilu is not None else 0,
                        fold_plan=fold[0] if fold else None, fold_blocks=fold[1] if fold else 0)
    check(lib.encdiff_groupnorm_bwd(C.byref(a), _s()), "encdiff_groupnorm_bwd")


LN_PARTS = 256  # fixed partial-row count of the LayerNorm backward (blocks without rows write zeros)


def layernorm_parts(rows, c):
    return LN_PARTS


def layernorm_fwd(x, gamma, beta, y, stats, eps=1e-5):
    rows, c = x.shape
    a = L.LayerNormArgs(rows=rows, c=c, eps=eps, x=_p(x), ldx=_ld(x), gamma=_p(gamma), beta=_p(beta),
                        y=_p(y), ldy=_ld(y), stats=_p(stats))
    check(lib.encdiff_layernorm_fwd(C.byref(a), _s()), "encdiff_layernorm_fwd")


def layernorm_bwd(x, gamma, stats, dy, dx, dgamma_part, dbeta_part, accumulate=False, ld_part=None, resid=None,
                  dy_from=None):
    """dx = LN_bwd(dy) (+ dx if accumulate) (+ resid: the residual-branch gradient, out of place).
    dy_from: as groupnorm_bwd."""
    rows, c = x.shape
    parts = layernorm_parts(rows, c)
    ld_part = c if ld_part is None else ld_part
    a = L.LayerNormArgs(rows=rows, c=c, eps=0.0, x=_p(x), ldx=_ld(x), gamma=_p(gamma), stats=_p(stats),
                        dy=_p(dy), lddy=_ld(dy), dx=_p(dx), lddx=_ld(dx), accumulate_dx=int(accumulate),
                        dgamma_part=_p(dgamma_part), dbeta_part=_p(dbeta_part), ld_part=ld_part, parts=parts,
                        resid=_p(resid), ld_resid=_ld(resid) if resid is not None else 0,
                        dy_from=None if dy_from is None else C.addressof(dy_from))
    check(lib.encdiff_layernorm_bwd(C.byref(a), _s()), "encdiff_layernorm_bwd")


# ------------------------------------------------------------------ attention
def attention_fwd(q, k, v, o, lse, batch, heads, sq, sk, dh, fp8=False):
    """fp8: scores on fp8 (e4m3) MFMA (configs[4]'s long-sequence level)."""
    a = L.AttnArgs(batch=batch, heads=heads, sq=sq, sk=sk, dh=dh, scale=dh ** -0.5,
                   q=_p(q), ldq=_ld(q), k=_p(k), ldk=_ld(k), v=_p(v), ldv=_ld(v), o=_p(o), ldo=_ld(o),
                   lse=_p(lse), fp8_qk=int(fp8))
    check(lib.encdiff_attention_fwd(C.byref(a), _s()), "encdiff_attention_fwd")


def attention_bwd(q, k, v, o, lse, d_o, dq, dk, dv, batch, heads, sq, sk, dh, fp8=False):
    a = L.AttnArgs(batch=batch, heads=heads, sq=sq, sk=sk, dh=dh, scale=dh ** -0.5,
                   q=_p(q), ldq=_ld(q), k=_p(k), ldk=_ld(k), v=_p(v), ldv=_ld(v), o=_p(o), ldo=_ld(o),
                   lse=_p(lse), d_o=_p(d_o), lddo=_ld(d_o), dq=_p(dq), lddq=_ld(dq), dk=_p(dk), lddk=_ld(dk),
                   dv=_p(dv), lddv=_ld(dv), fp8_qk=int(fp8))
    check(lib.encdiff_attention_bwd(C.byref(a), _s()), "encdiff_attention_bwd")


ST_TAIL_STATS_ADD = os.environ.get("ENCDIFF_ST_TAIL_STATS_ADD", "1") != "0"
# c = 64 tails on 32-row tiles too (the 16x16 level at B = 128: 1024 workgroups instead of 512):
# off -- 9.09 -> 9.13 ms/step (parity unchanged: test_graph_step_b128_matches_oracle with it on)
ST_TAIL_R32_C64 = os.environ.get("ENCDIFF_ST_TAIL_R32_C64", "0") != "0"


class StatSlots:
    """The producer-statistics slots an executor's transformer tails ADD into (two 32-row tiles
    per 64-row segment at 8x8): each must be zero before its one producer launch.  Outside a
    training step the fill runs right before the launch; a HipTrainer registers the slots seen
    (`register`) with its step prologue -- one zeroing launch per step -- and while a prologue step
    is active (`begin_step(True)`) the fills of exactly those views are skipped, each at most once
    per step (a second producer of one slot would add into a non-zero slot: asserted).  Keyed by
    (data pointer, shape, strides), so another view at the same address is never taken for one."""

    def __init__(self):
        self.seen = {}          # key -> view (every slot prepared since creation)
        self.prezeroed = set()  # keys the owner's step prologue zeroes
        self.prologue = False
        self._used = set()

    @staticmethod
    def key(v):
        return v.data_ptr(), tuple(v.shape), tuple(v.stride())

    def begin_step(self, prologue: bool):
        self.prologue = prologue
        self._used.clear()

    def prepare(self, view):
        k = self.key(view)
        if self.prologue and k in self.prezeroed:
            assert k not in self._used, "statistics slot produced twice in one prologue step"
            self._used.add(k)
            return
        view.zero_()
        self.seen[k] = view

    def register(self):
        """The views to zero in the step prologue (from now on their fills are skipped in steps)."""
        self.prezeroed.update(self.seen)
        return list(self.seen.values())


def st_tail_fwd(o1, t0, x, k2, v2, w, out, rows, c, tokens, heads, n_ctx, ln_eps, save=None,
                gn_stats=None, slots: Optional[StatSlots] = None, head=None) -> bool:
    """The row-local tail of a SpatialTransformer (attn1.to_out ... proj_out, attention.py:211-215,
    250-261) as one kernel.  w: dict of the bf16 GEMM weights / fp32 biases and LayerNorm affines
    (keys out1, b_out1, g2, be2, q2, out2, b_out2, g3, be3, ff1, b_ff1, ff2, b_ff2, po, b_po).
    save: None (inference) or a dict of the training activations (t1 n2 q2 o2 t2 n3 f a t3 s2 s3
    lse2).  head: None or (t2, n3): the kernel stops after norm3 and writes t2 and n3 = LN3(t2)
    there (bf16 rows), the feed-forward and proj_out being the caller's launches; in training with
    save = the nine activations up to norm3 (t1 n2 q2 o2 t2 n3 s2 s3 lse2; t2 / n3 the head rows).
    Returns False when the shape is outside the fused kernel's support (the caller issues the
    separate launches); any other error raises."""
    a = L.StTailArgs(rows=rows, c=c, tokens=tokens, heads=heads, n_ctx=n_ctx, ln_eps=ln_eps,
                     scale=(c // heads) ** -0.5,
                     o1=_p(o1), ld_o1=_ld(o1), t0=_p(t0), ld_t0=_ld(t0), x=_p(x), ld_x=_ld(x),
                     k2=_p(k2), v2=_p(v2), ld_kv=_ld(k2),
                     w_out1=_p(w["out1"]), ld_out1=_ld(w["out1"]), b_out1=_p(w["b_out1"]),
                     g2=_p(w["g2"]), be2=_p(w["be2"]), w_q2=_p(w["q2"]), ld_q2=_ld(w["q2"]),
                     w_out2=_p(w["out2"]), ld_out2=_ld(w["out2"]), b_out2=_p(w["b_out2"]),
                     g3=_p(w["g3"]), be3=_p(w["be3"]), w_ff1=_p(w["ff1"]), ld_ff1=_ld(w["ff1"]),
                     b_ff1=_p(w["b_ff1"]), w_ff2=_p(w["ff2"]), ld_ff2=_ld(w["ff2"]), b_ff2=_p(w["b_ff2"]),
                     w_po=_p(w["po"]), ld_po=_ld(w["po"]), b_po=_p(w["b_po"]), out=_p(out), ld_out=_ld(out))
    if save is not None:
        for k in ("t1", "n2", "q2", "o2", "t2", "n3", "f", "a", "t3", "s2", "s3", "lse2"):
            if k in save:
                setattr(a, "save_" + k, _p(save[k]))
        a.ld_save = _ld(save["t1"])
    if head is not None:
        # training (save): the nine activations up to norm3, t2 / n3 being the head rows
        assert gn_stats is None and (save is None or (save["t2"] is head[0] and save["n3"] is head[1]))
        a.head_t2, a.head_n3, a.ld_head = _p(head[0]), _p(head[1]), _ld(head[1])
        assert _ld(head[0]) == a.ld_head
    if gn_stats is not None:  # the next GroupNorm's producer statistics of out
        a.gn_stats, a.ld_gn_stats = _p(gn_stats), _ld(gn_stats)
        if ((c == 128 and rows // 64 < 256) or (c == 64 and ST_TAIL_R32_C64)) and ST_TAIL_STATS_ADD:
            # two 32-row tiles per 64-row segment add into the zeroed slots (twice the workgroups);
            # only this tensor's columns (the view may span a concat's other producer).  Inside a
            # training step whose prologue zeroes the registered slots (StatSlots) no fill runs.
            view = gn_stats[:, :c]
            if slots is not None:
                slots.prepare(view)
            else:
                view.zero_()
            a.gn_stats_add = 1
    rc = lib.encdiff_st_tail_fwd(C.byref(a), _s())
    if rc in (-2, -3):
        st_tail_fwd.declined = rc
        return False
    check(rc, "encdiff_st_tail_fwd")
    return True


def st_head_fwd(x, gn, w_in, b_in, g1, be1, w_qkv, t0, qkv, rows, c, tokens, gn_eps, ln_eps, in_stats=None,
                gn_gamma=None, gn_beta=None, gn_stats=None, n1=None, s1=None, self_stats=False) -> bool:
    """The row-local head of a SpatialTransformer (attention.py:250-254, 211) as one kernel:
    gn = GroupNorm32(x) from the producer's segment sums `in_stats` (self_stats: from x by the
    kernel itself, gn not written -- inference; else `gn` is read, already computed),
    t0 = proj_in(gn), n1 = LN1(t0) (saved with s1 when given), qkv = n1 Wqkv^T.
    Returns False outside the kernel's support (the caller issues the separate launches)."""
    a = L.StHeadArgs(rows=rows, c=c, tokens=tokens, gn_eps=gn_eps, ln_eps=ln_eps, x=_p(x), ld_x=_ld(x),
                     gn=_p(gn), ld_gn=_ld(gn), w_in=_p(w_in), ld_in=_ld(w_in), b_in=_p(b_in), g1=_p(g1), be1=_p(be1),
                     w_qkv=_p(w_qkv), ld_w_qkv=_ld(w_qkv), t0=_p(t0), ld_t0=_ld(t0), qkv=_p(qkv), ld_qkv=_ld(qkv))
    if self_stats:
        a.gn, a.ld_gn = None, 0
        a.gn_gamma, a.gn_beta = _p(gn_gamma), _p(gn_beta)
    elif in_stats is not None:
        a.gn_in_stats, a.ld_gn_in_stats = _p(in_stats), _ld(in_stats)
        a.gn_gamma, a.gn_beta, a.gn_stats = _p(gn_gamma), _p(gn_beta), _p(gn_stats)
    if n1 is not None:
        a.n1, a.ld_n1, a.s1 = _p(n1), _ld(n1), _p(s1)
    rc = lib.encdiff_st_head_fwd(C.byref(a), _s())
    if rc in (-2, -3):
        return False
    check(rc, "encdiff_st_head_fwd")
    return True


def st_tail_bwd_tile(c, rows, tokens) -> int:
    """The row tile encdiff_st_tail_bwd picks: tokens / tile dK2 / dV2 partial slabs per image."""
    return lib.encdiff_st_tail_bwd_tile(c, rows, tokens)


def st_tail_bwd(dy, save, wt, g3, g2, k2, v2, out, ln3, ln2, dk2, dv2, rows, c, tokens, heads, n_ctx,
                kv_part=None) -> bool:
    """Backward of the SpatialTransformer tail (encdiff_st_tail_bwd; attention.py:180-191, 206-215,
    226-232, 260-261): the input-gradient chain proj_out -> GEGLU FF -> norm3 -> attn2 (to_out,
    cross-attention to the concept tokens, to_q) -> norm2 -> attn1.to_out for row tiles in LDS.
    save: the forward's saved activations (f t2 t1 q2 o2 s3 s2 lse2); wt: the TRANSPOSED bf16
    weights (po ff2 ff1 out2 q2 out1, PackTable kind 6); out: d_t3 d_f d_t2 d_q2 d_t1 d_o1 (bf16);
    ln3 / ln2: (dgamma, dbeta) partial-row views [part_rows][c]; dk2 / dv2: the block's slices of
    the concept-token K / V gradient, written when a row tile holds a whole image; else kv_part
    (fp32 [rows/tile][n_ctx][2c]) receives per-tile partial slabs that st_head_bwd(kv=...) folds
    into dk2 / dv2.  False: shape not supported."""
    a = L.StTailBwdArgs(rows=rows, c=c, tokens=tokens, heads=heads, n_ctx=n_ctx, scale=(c // heads) ** -0.5,
                        part_rows=ln3[0].shape[0], dy=_p(dy), ld_dy=_ld(dy), f=_p(save["f"]), ld_f=_ld(save["f"]),
                        t2=_p(save["t2"]), t1=_p(save["t1"]), q2=_p(save["q2"]), o2=_p(save["o2"]),
                        ld_save=_ld(save["t2"]), s3=_p(save["s3"]), s2=_p(save["s2"]), lse2=_p(save["lse2"]),
                        k2=_p(k2), v2=_p(v2), ld_kv=_ld(k2),
                        w_po_t=_p(wt["po"]), w_ff2_t=_p(wt["ff2"]), w_ff1_t=_p(wt["ff1"]), w_out2_t=_p(wt["out2"]),
                        w_q2_t=_p(wt["q2"]), w_out1_t=_p(wt["out1"]), g3=_p(g3), g2=_p(g2),
                        d_t3=_p(out["d_t3"]), d_t2=_p(out["d_t2"]), d_q2=_p(out["d_q2"]), d_t1=_p(out["d_t1"]),
                        d_o1=_p(out["d_o1"]), ld_d=_ld(out["d_t3"]), d_f=_p(out["d_f"]), ld_df=_ld(out["d_f"]),
                        ln3_dg=_p(ln3[0]), ln3_db=_p(ln3[1]), ln2_dg=_p(ln2[0]), ln2_db=_p(ln2[1]),
                        ld_part=_ld(ln3[0]), dk2=_p(dk2), dv2=_p(dv2), ld_dkv=_ld(dk2), kv_part=_p(kv_part))
    for k in ("d_t2", "d_q2", "d_t1", "d_o1"):
        assert _ld(out[k]) == a.ld_d, k
    for k in ("t1", "q2", "o2"):
        assert _ld(save[k]) == a.ld_save, k
    assert _ld(v2) == a.ld_kv and _ld(dv2) == a.ld_dkv
    assert all(_ld(t) == a.ld_part for t in (ln3[1], ln2[0], ln2[1]))
    assert ln2[0].shape[0] == a.part_rows
    rc = lib.encdiff_st_tail_bwd(C.byref(a), _s())
    if rc in (-2, -3):
        return False
    check(rc, "encdiff_st_tail_bwd")
    return True


def st_head_bwd(d_qkv, d_t1, t0, s1, g1, w_qkv_t, w_in_t, d_t0, d_gn, ln1, rows, c, kv=None) -> bool:
    """Backward of the SpatialTransformer head after the self-attention backward
    (encdiff_st_head_bwd; attention.py:211 norm1 + attn1 q/k/v, :253-254 proj_in):
    d_n1 = d_qkv Wqkv, d_t0 = d_t1 + LN1'(t0; d_n1), d_gn = d_t0 Win (transposed bf16 weights);
    ln1: (dgamma, dbeta) partial-row views.  kv = (kv_part, tiles per image, n_ctx, batch, dk2, dv2):
    the tail's dK2 / dV2 partial slabs folded in tile order by the same grid.  False: shape not
    supported."""
    a = L.StHeadBwdArgs(rows=rows, c=c, part_rows=ln1[0].shape[0], d_qkv=_p(d_qkv), ld_dqkv=_ld(d_qkv),
                        d_t1=_p(d_t1), ld_dt1=_ld(d_t1), t0=_p(t0), ld_t0=_ld(t0), s1=_p(s1), g1=_p(g1),
                        w_qkv_t=_p(w_qkv_t), w_in_t=_p(w_in_t), d_t0=_p(d_t0), ld_dt0=_ld(d_t0), d_gn=_p(d_gn),
                        ld_dgn=_ld(d_gn), ln1_dg=_p(ln1[0]), ln1_db=_p(ln1[1]), ld_part=_ld(ln1[0]))
    if kv is not None:
        a.kv_part, a.kv_tiles, a.n_ctx, a.batch = _p(kv[0]), kv[1], kv[2], kv[3]
        a.dk2, a.dv2, a.ld_dkv = _p(kv[4]), _p(kv[5]), _ld(kv[4])
        assert _ld(kv[5]) == a.ld_dkv
    assert _ld(ln1[1]) == a.ld_part
    rc = lib.encdiff_st_head_bwd(C.byref(a), _s())
    if rc in (-2, -3):
        return False
    check(rc, "encdiff_st_head_bwd")
    return True


STWG_PROBS = {}  # host blob address of a planned StWgrad launch -> its problems as GemmArgs (bench.py's record)


class StWgrad:
    """The weight gradients of a fused transformer block's Linear layers (encdiff_st_wgrad_*: one
    grid of large output blocks + a chunk fold), planned once per distinct problem list (the
    executor's buffers are static per batch size) and kept for the life of the object: captured
    graphs read the device description at replay.  Slabs live in a scratch of their own
    (STWG_WS_FLOATS), not in the split-K workspace halves."""

    def __init__(self):
        self._plans = {}

    def launch(self, probs, ride=False):
        """probs: [(dy [K][M], x [K][N], dw [M][N] fp32 (+=), db [M] fp32 or None)].
        ride=True: only the weight-gradient grid is launched; returns (device plan, fold blocks) for
        the next GroupNorm backward to carry (groupnorm_bwd(fold=)), or None when there is no fold
        (every problem in one chunk).  The fold must be launched before the gradients are read."""
        arr = (L.WgradProb * len(probs))(*[
            L.WgradProb(dy=_p(dy), ld_dy=_ld(dy), x=_p(x), ld_x=_ld(x), dw=_p(dw), ld_dw=_ld(dw), db=_p(db),
                        M=dy.shape[1], N=x.shape[1], K=dy.shape[0])
            for dy, x, dw, db in probs])
        key = bytes(arr)
        ent = self._plans.get(key)
        if ent is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("encdiff_st_wgrad first planned inside a graph capture: run an eager step first")
            ws = scratch("stwg_ws", STWG_WS_FLOATS).data_ptr()
            nb = C.c_long(0)
            check(lib.encdiff_st_wgrad_plan(arr, len(probs), ws, STWG_WS_FLOATS, None, 0, C.byref(nb)),
                  "encdiff_st_wgrad_plan")
            host = (C.c_longlong * ((nb.value + 7) // 8))()
            check(lib.encdiff_st_wgrad_plan(arr, len(probs), ws, STWG_WS_FLOATS, C.addressof(host), C.sizeof(host),
                                            C.byref(nb)), "encdiff_st_wgrad_plan")
            dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(torch.cuda.current_device())
            gem = [L.GemmArgs(M=q.M, N=q.N, K=q.K, a_mode=L.OPA_ROWM, b_mode=L.OPB_ROWN, c_mode=L.OUT_F32_ACCUM,
                              a=q.dy, lda=q.ld_dy, b=q.x, ldb=q.ld_x, c=q.dw, ldc=q.ld_dw, split_k=1) for q in arr]
            ent = self._plans[key] = (host, dev)
            STWG_PROBS[C.addressof(host)] = gem
        if not ride:
            check(lib.encdiff_st_wgrad_launch(C.addressof(ent[0]), ent[1].data_ptr(), _s()), "encdiff_st_wgrad_launch")
            return None
        plan, nb = C.c_void_p(), C.c_int(0)
        check(lib.encdiff_st_wgrad_launch_nofold(C.addressof(ent[0]), ent[1].data_ptr(), _s(), C.byref(plan),
                                                 C.byref(nb)), "encdiff_st_wgrad_launch_nofold")
        return (plan.value, nb.value) if nb.value > 0 else None


def whole_wgrad_args(dy, x, dw, db=None):
    """linear_wgrad's problem (dw += dy^T x, db += sum dy) as ONE whole GEMM description (split-K
    1, no slabs) for a WgradGroup: the group kernel chunks it itself."""
    return _whole_wgrad(lambda off: linear_wgrad_args(dy, x, dw, db, off))


RC_TILE_M = int(os.environ.get("ENCDIFF_RC_TILE_M", "0"))  # plan overrides for tuning (0: heuristic)
RC_TILE_N = int(os.environ.get("ENCDIFF_RC_TILE_N", "0"))


def resconv_supported(x, g: Geom, w, resample=L.RESAMPLE_NONE, film=None, ld_film=0, cskip=0, groups=32) -> bool:
    """Whether encdiff_resconv_fwd plans this conv (encdiff_resconv_query: shapes, LDS fit, FiLM
    row alignment), so a caller can choose the fused pair before launching either of its convs."""
    if g.h != g.w:
        return False
    fp = _p(film) or 0
    key = (g.batch, g.h, w.shape[1] // 9, w.shape[0], resample, groups, _ld(x), _ld(w), RC_TILE_M, RC_TILE_N,
           fp % 16 if film is not None else -1, ld_film % 4, cskip)
    hit = _RC_OK.get(key)
    if hit is None:
        a = L.ResConvArgs(batch=g.batch, h=g.h, cin=w.shape[1] // 9, cout=w.shape[0], resample=resample,
                          groups=groups, x=_p(x), ld_x=_ld(x), gamma=_p(x), beta=_p(x), film=fp or None,
                          ld_film=ld_film, w=_p(w), ld_w=_ld(w), y=_p(x), ld_y=w.shape[0], cskip=cskip,
                          xskip=_p(x) if cskip else None, ld_xskip=cskip, wskip=_p(w) if cskip else None,
                          ld_wskip=cskip, tile_m=RC_TILE_M, tile_n=RC_TILE_N)
        hit = _RC_OK[key] = lib.encdiff_resconv_query(C.byref(a), None, None) == 0
    return hit


_RC_OK = {}
_RC_Q = {}  # resconv_fwd(query=True): argument bytes -> planned


def resconv_fwd(x, g: Geom, w, y, gamma, beta, eps, silu=True, film=None, ld_film=0, bias=None,
                resample=L.RESAMPLE_NONE, resid=None, resid_resample=L.RESAMPLE_NONE, xskip=None, wskip=None,
                bskip=None, groups=32, query=False) -> bool:
    """An inference ResBlock conv with the GroupNorm in front of it, one launch
    (openaimodel_enc.py:255-275): y = conv3x3(resample(SiLU(GN(x)(1 + scale) + shift))) + bias
    + resid (read through resid_resample) or bf16(xskip wskip^T + bskip).  x: [B*h*h][cin] at the
    geometry g, w: packed [cout][9*cin].  Returns False outside the kernel's support (the caller
    issues the unfused launches).  query=True: nothing launched -- whether the launch with exactly
    these arguments would be planned (encdiff_resconv_query, memoised on the argument bytes), so a
    caller can commit to a pair of launches before issuing the first."""
    cin = w.shape[1] // 9
    a = L.ResConvArgs(batch=g.batch, h=g.h, cin=cin, cout=w.shape[0], resample=resample, groups=groups,
                      silu=int(silu), eps=eps, x=_p(x), ld_x=_ld(x), gamma=_p(gamma), beta=_p(beta),
                      film=_p(film), ld_film=ld_film, w=_p(w), ld_w=_ld(w), bias=_p(bias), y=_p(y), ld_y=_ld(y),
                      tile_m=RC_TILE_M, tile_n=RC_TILE_N)
    if resid is not None:
        a.resid, a.ld_resid, a.resid_resample = _p(resid), _ld(resid), resid_resample
    if xskip is not None:
        a.cskip, a.xskip, a.ld_xskip = xskip.shape[1], _p(xskip), _ld(xskip)
        a.wskip, a.ld_wskip, a.bskip = _p(wskip), _ld(wskip), _p(bskip)
    if query:
        key = bytes(a)
        hit = _RC_Q.get(key)
        if hit is None:
            hit = _RC_Q[key] = lib.encdiff_resconv_query(C.byref(a), None, None) == 0
        return hit
    rc = lib.encdiff_resconv_fwd(C.byref(a), _s())
    if rc in (-2, -3):
        return False
    check(rc, "encdiff_resconv_fwd")
    return True


# ------------------------------------------------------------------ elementwise
def ew(op, x, y, x2=None, rows=None, cols=None, accumulate=False, resample=0, g: Optional[Geom] = None):
    rows = rows if rows is not None else y.shape[0]
    cols = cols if cols is not None else y.shape[1]
    a = L.EwArgs(op=op, rows=rows, cols=cols, x=_p(x), ldx=_ld(x), x2=_p(x2), ldx2=_ld(x2) if x2 is not None else 0,
                 y=_p(y), ldy=_ld(y), accumulate=int(accumulate), resample=resample,
                 batch=g.batch if g else 0, h=g.h if g else 0, w=g.w if g else 0)
    check(lib.encdiff_elementwise(C.byref(a), _s()), "encdiff_elementwise")


def geglu_fwd(f, y):
    ew(L.EW_GEGLU, f, y, cols=y.shape[1])


def geglu_bwd(f, dy, df):
    ew(L.EW_GEGLU_BWD, f, df, x2=dy, rows=dy.shape[0], cols=dy.shape[1])


def resample(x, y, g_out: Geom, mode, accumulate=False):
    ew(L.EW_RESAMPLE, x, y, resample=mode, g=g_out, accumulate=accumulate)


def resample_bwd(dy, dx, g_src: Geom, mode, accumulate=False):
    """dx (at the forward source resolution g_src) (+)= adjoint of `mode` applied to dy."""
    ew(L.EW_RESAMPLE_BWD, dy, dx, resample=mode, g=g_src, accumulate=accumulate)


def small_conv_in_fwd(x_nchw, g: Geom, weight, bias, y):
    cout, cin = weight.shape[0], weight.shape[1]
    a = L.SmallConvArgs(batch=g.batch, h=g.h, w=g.w, cin=cin, cout=cout, x=_p(x_nchw), ldx=0, x_f32=1,
                        weight=_p(weight), bias=_p(bias), y=_p(y), ldy=_ld(y), y_f32=0)
    check(lib.encdiff_small_conv_fwd(C.byref(a), _s()), "encdiff_small_conv_fwd")


def small_conv_in_wgrad(x_nchw, g: Geom, weight, dy, dweight, dbias):
    cout, cin = weight.shape[0], weight.shape[1]
    a = L.SmallConvArgs(batch=g.batch, h=g.h, w=g.w, cin=cin, cout=cout, x=_p(x_nchw), x_f32=1,
                        weight=_p(weight), dy=_p(dy), lddy=_ld(dy), dy_f32=0, dweight=_p(dweight), dbias=_p(dbias))
    check(lib.encdiff_small_conv_bwd(C.byref(a), _s()), "encdiff_small_conv_bwd(in)")


def small_conv_out_fwd(x, g: Geom, weight, bias, y_nchw):
    cout, cin = weight.shape[0], weight.shape[1]
    a = L.SmallConvArgs(batch=g.batch, h=g.h, w=g.w, cin=cin, cout=cout, x=_p(x), ldx=_ld(x), x_f32=0,
                        weight=_p(weight), bias=_p(bias), y=_p(y_nchw), ldy=0, y_f32=1)
    check(lib.encdiff_small_conv_fwd(C.byref(a), _s()), "encdiff_small_conv_fwd")


def nchw_to_rows(x, cpad, y):
    """fp32 NCHW [B][C][H][W] -> bf16 rows [B*H*W][cpad] (channels C..cpad-1 zero)."""
    B, Cc, H, W = x.shape
    assert x.is_contiguous() and x.dtype == F32 and y.shape == (B * H * W, cpad)
    check(lib.encdiff_nchw_to_rows(_p(x), B, Cc, H * W, cpad, _p(y), _ld(y), _s()), "encdiff_nchw_to_rows")


def pack_conv_pad8(w):
    """[co][ci][3][3] (ci <= 8) -> bf16 [co][9*8] with zero channels ci..7 (the GEMM B layout of
    a 3x3 conv over channel-padded rows)."""
    co, ci = w.shape[0], w.shape[1]
    out = torch.zeros(co, 3, 3, 8, device=w.device, dtype=F32)
    out[..., :ci] = w.detach().float().permute(0, 2, 3, 1)
    return out.reshape(co, 72).to(BF16).contiguous()


def small_conv_out_bwd(x, g: Geom, weight, dy_nchw, dx, dweight, dbias):
    cout, cin = weight.shape[0], weight.shape[1]
    a = L.SmallConvArgs(batch=g.batch, h=g.h, w=g.w, cin=cin, cout=cout, x=_p(x), ldx=_ld(x), x_f32=0,
                        weight=_p(weight), dy=_p(dy_nchw), lddy=0, dy_f32=1, dx=_p(dx),
                        lddx=_ld(dx) if dx is not None else 0, dweight=_p(dweight), dbias=_p(dbias))
    check(lib.encdiff_small_conv_bwd(C.byref(a), _s()), "encdiff_small_conv_bwd(out)")


# ------------------------------------------------------------------ diffusion / optimizer
def timestep_embedding(t, dim, out, max_period=10000.0):
    check(lib.encdiff_timestep_embedding(_p(t), t.shape[0], dim, max_period, _p(out), _s()),
          "encdiff_timestep_embedding")


def q_sample(x0, eps, t, sqrt_ac, sqrt_1mac, xt, x0_scale=None):
    """x_t = sqrt_ac[t] x0 + sqrt_1mac[t] eps; x0_scale (device scalar): x0 := x0_scale * x0."""
    b = x0.shape[0]
    if x0_scale is not None:
        check(lib.encdiff_q_sample_scaled(_p(x0), _p(x0_scale), _p(eps), _p(t), _p(sqrt_ac), _p(sqrt_1mac), b,
                                          x0.numel() // b, _p(xt), _s()), "encdiff_q_sample_scaled")
        return
    check(lib.encdiff_q_sample(_p(x0), _p(eps), _p(t), _p(sqrt_ac), _p(sqrt_1mac), b, x0.numel() // b, _p(xt),
                               _s()), "encdiff_q_sample")


def l1_loss(pred, eps, t, lvlb, out2, grad=None, l_simple_weight=1.0):
    """out2 = (loss, loss_vlb); grad = the L1 seed.  Per-sample partials and the last-block
    ticket live in the device's library scratch (see `scratch`; the ticket returns to zero)."""
    b = pred.shape[0]
    part = scratch("l1_partials", b, torch.float32, pred.device.index)
    tick = scratch("l1_ticket", 1, torch.int32, pred.device.index)
    check(lib.encdiff_l1_loss(_p(pred), _p(eps), _p(t), _p(lvlb), b, pred.numel() // b, l_simple_weight,
                              _p(out2), _p(grad), _p(part), _p(tick), _s()), "encdiff_l1_loss")


def ddim_step(x, e, noise, a_t, a_prev, sigma, s1, x_prev, pred_x0=None):
    check(lib.encdiff_ddim_step(_p(x), _p(e), _p(noise), x.numel(), float(a_t), float(a_prev), float(sigma),
                                float(s1), _p(x_prev), _p(pred_x0), _s()), "encdiff_ddim_step")


def ddim_step_indexed(x, e, noise, coef, index, x_prev, pred_x0=None, advance=True):
    check(lib.encdiff_ddim_step_indexed(_p(x), _p(e), _p(noise), x.numel(), _p(coef), _p(index), int(advance),
                                        _p(x_prev), _p(pred_x0), _s()), "encdiff_ddim_step_indexed")


def adamw_ema(p, g, m, v, hyper, ema=None, ema_n=0, mirror=None):
    """mirror: bf16 buffer of p's size that receives the updated weights (arena.mirror)."""
    check(lib.encdiff_adamw_ema_mirror(_p(p), _p(g), _p(m), _p(v), _p(ema), p.numel(), _p(hyper), ema_n, _p(mirror),
                                       _s()), "encdiff_adamw_ema_mirror")


def adamw_hyper(lr, step, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, ema_one_minus_decay=0.0):
    """Host-side (float64) scalars exactly as torch.optim.AdamW computes them."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    return [lr, beta1, beta2, eps, weight_decay, lr / bc1, 1.0 / math.sqrt(bc2), ema_one_minus_decay]


def pack_weights(src_f32, dst_bf16, jobs_dev, njobs):
    check(lib.encdiff_pack_weights(_p(src_f32), _p(dst_bf16), _p(jobs_dev), njobs, _s()), "encdiff_pack_weights")


def grad_fold(dw, co, cin, cpad, taps, gw, db=None, gb=None):
    """gw[o][c][t] += dw[o][t][c] (dw rows [taps][cpad]); gb += db, db zeroed (encdiff_grad_fold)."""
    assert dw.dtype == F32 and gw.dtype == F32 and gw.is_contiguous() and gw.numel() == co * cin * taps
    assert dw.is_contiguous() and dw.numel() >= co * taps * cpad
    check(lib.encdiff_grad_fold(_p(dw), co, cin, cpad, taps, _p(db), _p(gw), _p(gb), _s()), "encdiff_grad_fold")


def reduce_partials(part, ld, rows, cols, col_index, grad):
    check(lib.encdiff_reduce_partials(_p(part), ld, rows, cols, _p(col_index), _p(grad), _s()),
          "encdiff_reduce_partials")


class StepPrologue:
    """ONE launch in front of a training step (encdiff_step_prologue): zero the registered byte
    regions (the gradient arena, producer-statistics slots that the step's kernels add into),
    draw t ~ U{0..T-1} and noise ~ N(0, 1) with Philox4x32-10 from a device counter, advance that
    counter and (optionally) the image pool's epoch step.  Replaces torch.randint / randn_like
    (ddpm_enc.py:1041, :1184), the arena grad.zero_() and the pool's counter increment.  The job
    table lives in device memory; call `set_jobs` whenever the regions change (not during capture)."""

    def __init__(self, dev, seed: int):
        self.dev = torch.device(dev)
        self.seed = int(seed) & ((1 << 64) - 1)
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.done = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.jobs_dev = None
        self.njobs = 0
        self._keep = []

    def set_jobs(self, regions):
        """regions: 2-D (or 1-D) tensor views to zero; row bytes and strides multiples of 16 B."""
        jobs = []
        self._keep = list(regions)
        for r in regions:
            r2 = r.view(1, -1) if r.dim() == 1 else r
            assert r2.dim() == 2 and r2.stride(1) == 1, "zero job: 2-D rows with unit column stride"
            es = r2.element_size()
            rb, ld = r2.shape[1] * es, r2.stride(0) * es
            assert rb % 16 == 0 and ld % 16 == 0 and r2.data_ptr() % 16 == 0, "zero job: 16-byte multiples"
            jobs.append(L.ZeroJob(ptr=r2.data_ptr(), rows=r2.shape[0], row_bytes=rb, ld_bytes=ld))
        n = len(jobs)
        raw = bytearray(C.sizeof(L.ZeroJob) * max(n, 1))
        for i, j in enumerate(jobs):
            C.memmove((C.c_char * C.sizeof(L.ZeroJob)).from_buffer(raw, i * C.sizeof(L.ZeroJob)), C.byref(j),
                       C.sizeof(L.ZeroJob))
        self.jobs_dev = torch.frombuffer(raw, dtype=torch.uint8).to(self.dev)
        self.njobs = n

    def __call__(self, t=None, noise=None, timesteps=1000, data_step=None):
        a = L.StepPrologueArgs(jobs=_p(self.jobs_dev), njobs=self.njobs, batch=t.numel() if t is not None else 0,
                               timesteps=timesteps, seed=self.seed, rng_counter=_p(self.counter),
                               data_step=_p(data_step), t=_p(t), noise=_p(noise),
                               n_noise=noise.numel() if noise is not None else 0, done=_p(self.done))
        if t is not None:
            assert t.dtype == torch.int64 and t.is_contiguous()
        if noise is not None:
            assert noise.dtype == F32 and noise.is_contiguous()
        check(lib.encdiff_step_prologue(C.byref(a), _s()), "encdiff_step_prologue")


def gather_images_u8(pool_u8, perm, step, batch, out, advance=True):
    """Batch gather from the HBM-resident uint8 dataset + ToTensor/Normalize/CHW
    (disdata.py:82-88, ddpm_enc.py:347-353) -> out fp32 [batch][c][h][w]."""
    n, h, w, c = pool_u8.shape
    assert pool_u8.is_cuda and perm.is_cuda and step.is_cuda and out.is_cuda, "HIP device tensors required"
    assert pool_u8.dtype == torch.uint8 and pool_u8.is_contiguous() and out.is_contiguous()
    assert out.shape == (batch, c, h, w) and out.dtype == torch.float32
    spe = perm.numel() // batch
    check(lib.encdiff_gather_images_u8(_p(pool_u8), n, h, w, c, _p(perm), _p(step), spe, batch, int(advance),
                                       _p(out), _s()), "encdiff_gather_images_u8")


def encoder_warp_fwd(u, params, unit_stride, units, context_dim, out):
    """Encoder4.warp forward (openaimodel_enc.py:1015-1041) -> out fp32 [B, units*context_dim]."""
    assert u.is_cuda and params.is_cuda and out.is_cuda, "HIP device tensors required"
    check(lib.encdiff_encoder_warp_fwd(_p(u), u.stride(0), u.shape[0], units, _p(params), unit_stride, context_dim,
                                       _p(out), out.stride(0), _s()), "encdiff_encoder_warp_fwd")


_WARP_SCRATCH = {}
_RETIRED = []  # outgrown scratch stays allocated: graphs captured earlier still address it


def encoder_warp_bwd(u, params, unit_stride, units, context_dim, dout, du, grads):
    """Backward of the warp MLPs: du, and the weight gradients ADDED into `grads` (per-chunk
    partials in a cached scratch, folded in order)."""
    assert dout.stride(1) == 1 and du.stride(1) == 1
    n = lib.encdiff_encoder_warp_partials_floats(u.shape[0], units, unit_stride)
    key = (u.device.index, n)
    part = _WARP_SCRATCH.get(key)
    if part is None:
        part = _WARP_SCRATCH[key] = torch.empty(max(n, 1), device=u.device, dtype=torch.float32)
    check(lib.encdiff_encoder_warp_bwd(_p(u), u.stride(0), u.shape[0], units, _p(params), unit_stride, context_dim,
                                       _p(dout), dout.stride(0), _p(du), du.stride(0), _p(grads), _p(part), _s()),
          "encdiff_encoder_warp_bwd")


# ------------------------------------------------------------------ fp32 (ENCDIFF_DT_F32) forward
# The reference-precision forms of the same entry points (include/encdiff_hip.h "dtype"): fp32
# activations end to end, for the fp32 parity path (unet_f32.py).
def _f32(t):
    assert t.dtype == F32, "fp32 operand expected"
    return t


def gemm_f32(M, N, K, a, lda, b, ldb, c, ldc, *, a_mode=L.OPA_ROWK, b_mode=L.OPB_ROWK,
             conv: Optional[L.ConvGeom] = None, bias=None, resid=None, accumulate=False, alpha=1.0, conv_cout=0,
             bias_grad=None):
    args = L.GemmArgs(M=M, N=N, K=K, a_mode=a_mode, b_mode=b_mode,
                      c_mode=L.OUT_F32_ACCUM if accumulate else L.OUT_F32, a=_p(_f32(a)), lda=lda, b=_p(_f32(b)),
                      ldb=ldb, c=_p(_f32(c)), ldc=ldc, conv=conv if conv is not None else L.ConvGeom(), alpha=alpha,
                      split_k=1, bias=_p(bias), resid=_p(resid), ld_resid=_ld(resid) if resid is not None else 0,
                      conv_cout=conv_cout, bias_grad=_p(bias_grad), dtype=L.DT_F32)
    check(lib.encdiff_gemm(C.byref(args), _s()), "encdiff_gemm(fp32)")


# ---- fp32 backward (the reference-precision gradient path, unet_f32.py)
def linear_dgrad_f32(dy, w, dx, accumulate=False):
    """dx[M][K] (+)= dy[M][N] w[N][K] (the input gradient of y = x w^T)."""
    M, N = dy.shape
    gemm_f32(M, w.shape[1], N, dy, _ld(dy), w, _ld(w), dx, _ld(dx), b_mode=L.OPB_ROWN, accumulate=accumulate)


def linear_wgrad_f32(dy, x, dw, db=None):
    """dw[N][K] += dy^T x, db[N] += column sums of dy (accumulated into arena gradients)."""
    M, N = dy.shape
    gemm_f32(N, x.shape[1], M, dy, _ld(dy), x, _ld(x), dw, _ld(dw), a_mode=L.OPA_ROWM, b_mode=L.OPB_ROWN,
             accumulate=True, bias_grad=db)


def conv3x3_dgrad_f32(dy, g: Geom, w, dx, accumulate=False):
    """dx[pixels][cin] (+)= conv3x3^T(dy) at the conv resolution; w [cout][9*cin] tap-major."""
    cout, cin = w.shape[0], w.shape[1] // 9
    gemm_f32(g.pixels, cin, 9 * cout, dy, 0, w, _ld(w), dx, _ld(dx), a_mode=L.OPA_IM2COL,
             b_mode=L.OPB_CONV_DGRAD, conv=L.ConvGeom(batch=g.batch, h=g.h, w=g.w, cin=cout, resample=0,
                                                      ld_src=_ld(dy)), conv_cout=cout, accumulate=accumulate)


def conv3x3_wgrad_f32(dy, x, g: Geom, cin, dw, db=None, resample=0):
    """dw[cout][9*cin] += dy^T im2col(resample(x)) (channels-last taps), db += column sums of dy."""
    cout = dy.shape[1]
    gemm_f32(cout, 9 * cin, g.pixels, dy, _ld(dy), x, _ld(x), dw, _ld(dw), a_mode=L.OPA_ROWM, b_mode=L.OPB_IM2COL,
             conv=L.ConvGeom(batch=g.batch, h=g.h, w=g.w, cin=cin, resample=resample, ld_src=_ld(x)),
             accumulate=True, bias_grad=db)


def groupnorm_bwd_f32(x, g: Geom, gamma, beta, stats, silu, dy, dx, dgamma_part, dbeta_part, ld_part, film=None,
                      ld_film=0, dfilm=None, ld_dfilm=0, accumulate=False, resid=None, groups=32):
    c = x.shape[1]
    a = L.GroupNormArgs(batch=g.batch, hw=g.h * g.w, c=c, groups=groups, silu=int(silu), x=_p(_f32(x)), ldx=_ld(x),
                        gamma=_p(gamma), beta=_p(beta), film=_p(film), ld_film=ld_film, stats=_p(stats),
                        dy=_p(_f32(dy)), lddy=_ld(dy), dx=_p(_f32(dx)), lddx=_ld(dx), accumulate_dx=int(accumulate),
                        dgamma_part=_p(dgamma_part), dbeta_part=_p(dbeta_part), ld_part=ld_part, dfilm=_p(dfilm),
                        ld_dfilm=ld_dfilm, resid=_p(resid), ld_resid=_ld(resid) if resid is not None else 0,
                        dtype=L.DT_F32)
    check(lib.encdiff_groupnorm_bwd(C.byref(a), _s()), "encdiff_groupnorm_bwd(fp32)")


def layernorm_bwd_f32(x, gamma, stats, dy, dx, dgamma_part, dbeta_part, parts, ld_part, accumulate=False,
                      resid=None):
    rows, c = x.shape
    a = L.LayerNormArgs(rows=rows, c=c, x=_p(_f32(x)), ldx=_ld(x), gamma=_p(gamma), stats=_p(stats),
                        dy=_p(_f32(dy)), lddy=_ld(dy), dx=_p(_f32(dx)), lddx=_ld(dx), accumulate_dx=int(accumulate),
                        dgamma_part=_p(dgamma_part), dbeta_part=_p(dbeta_part), ld_part=ld_part, parts=parts,
                        resid=_p(resid), ld_resid=_ld(resid) if resid is not None else 0, dtype=L.DT_F32)
    check(lib.encdiff_layernorm_bwd(C.byref(a), _s()), "encdiff_layernorm_bwd(fp32)")


def attention_bwd_f32(q, k, v, o, lse, d_o, dq, dk, dv, batch, heads, sq, sk, dh):
    a = L.AttnArgs(batch=batch, heads=heads, sq=sq, sk=sk, dh=dh, scale=dh ** -0.5,
                   q=_p(_f32(q)), ldq=_ld(q), k=_p(_f32(k)), ldk=_ld(k), v=_p(_f32(v)), ldv=_ld(v),
                   o=_p(_f32(o)), ldo=_ld(o), lse=_p(lse), d_o=_p(_f32(d_o)), lddo=_ld(d_o), dq=_p(_f32(dq)),
                   lddq=_ld(dq), dk=_p(_f32(dk)), lddk=_ld(dk), dv=_p(_f32(dv)), lddv=_ld(dv), dtype=L.DT_F32)
    check(lib.encdiff_attention_bwd(C.byref(a), _s()), "encdiff_attention_bwd(fp32)")


def linear_f32(x, w, y, bias=None, resid=None):
    """y[M][N] = x[M][K] w[N][K]^T (+bias)(+resid), fp32 rows."""
    M, K = x.shape
    N = w.shape[0]
    gemm_f32(M, N, K, x, _ld(x), w, _ld(w), y, _ld(y), bias=bias, resid=resid)


def conv3x3_f32(x, g: Geom, cin, w, y, bias=None, resid=None, resample=0):
    """3x3 conv (pad 1) of fp32 NHWC rows; w [cout][9*cin] (tap-major, channel inner); resample
    NONE or UP2 (nearest x2 read through the im2col gather, g = the output geometry)."""
    gemm_f32(g.pixels, w.shape[0], 9 * cin, x, 0, w, _ld(w), y, _ld(y), a_mode=L.OPA_IM2COL,
             conv=L.ConvGeom(batch=g.batch, h=g.h, w=g.w, cin=cin, resample=resample, ld_src=_ld(x)),
             bias=bias, resid=resid)


def groupnorm_f32(x, g: Geom, gamma, beta, y, stats, eps, silu, film=None, ld_film=0, groups=32):
    a = L.GroupNormArgs(batch=g.batch, hw=g.h * g.w, c=x.shape[1], groups=groups, eps=eps, silu=int(silu),
                        x=_p(_f32(x)), ldx=_ld(x), gamma=_p(gamma), beta=_p(beta), film=_p(film), ld_film=ld_film,
                        y=_p(_f32(y)), ldy=_ld(y), stats=_p(stats), dtype=L.DT_F32)
    check(lib.encdiff_groupnorm_fwd(C.byref(a), _s()), "encdiff_groupnorm_fwd(fp32)")


def layernorm_f32(x, gamma, beta, y, eps=1e-5, stats=None):
    rows, c = x.shape
    a = L.LayerNormArgs(rows=rows, c=c, eps=eps, x=_p(_f32(x)), ldx=_ld(x), gamma=_p(gamma), beta=_p(beta),
                        y=_p(_f32(y)), ldy=_ld(y), stats=_p(stats), dtype=L.DT_F32)
    check(lib.encdiff_layernorm_fwd(C.byref(a), _s()), "encdiff_layernorm_fwd(fp32)")


def attention_f32(q, k, v, o, batch, heads, sq, sk, dh, lse=None):
    a = L.AttnArgs(batch=batch, heads=heads, sq=sq, sk=sk, dh=dh, scale=dh ** -0.5,
                   q=_p(_f32(q)), ldq=_ld(q), k=_p(_f32(k)), ldk=_ld(k), v=_p(_f32(v)), ldv=_ld(v),
                   o=_p(_f32(o)), ldo=_ld(o), lse=_p(lse), dtype=L.DT_F32)
    check(lib.encdiff_attention_fwd(C.byref(a), _s()), "encdiff_attention_fwd(fp32)")


def ew_f32(op, x, y, x2=None, rows=None, cols=None, accumulate=False, resample=0, g: Optional[Geom] = None):
    rows = rows if rows is not None else y.shape[0]
    cols = cols if cols is not None else y.shape[1]
    a = L.EwArgs(op=op, rows=rows, cols=cols, x=_p(_f32(x)), ldx=_ld(x), x2=_p(x2),
                 ldx2=_ld(x2) if x2 is not None else 0, y=_p(_f32(y)), ldy=_ld(y), accumulate=int(accumulate),
                 resample=resample, batch=g.batch if g else 0, h=g.h if g else 0, w=g.w if g else 0, dtype=L.DT_F32)
    check(lib.encdiff_elementwise(C.byref(a), _s()), "encdiff_elementwise(fp32)")


def timestep_embedding_f32(t, dim, out, max_period=10000.0):
    check(lib.encdiff_timestep_embedding_f32(_p(t), t.shape[0], dim, max_period, _p(_f32(out)), _s()),
          "encdiff_timestep_embedding_f32")


def nchw_rows_f32(x, batch, c, hw, cpad, y, ld, to_rows=True):
    check(lib.encdiff_nchw_rows_f32(_p(_f32(x)), batch, c, hw, cpad, _p(_f32(y)), ld, 0 if to_rows else 1, _s()),
          "encdiff_nchw_rows_f32")
