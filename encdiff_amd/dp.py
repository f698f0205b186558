"""Data-parallel exchange of the EncDiff training step.

The step is pure data parallel: each rank draws its own batch and noise (seed 1234+rank),
runs the full step on its GPU, and the ONLY exchange is the mean of the gradients of the
38.84 M trainable parameters (UNet + Encoder4), which AdamW needs identical on every rank
(the reference gets the same from Lightning DDP, ddpm_enc.py:1598-1639 + main_val.py).

The gradient arena (`arena.ParamArena.grad`, one flat fp32 buffer) is split into
contiguous buckets in the order their gradients become final inside the step (three with the
split backward, `UNetExecutor.split_plan`):
  bucket 0 = [0, lo): the UNet parameters before the output blocks (17.40 M params, final when
             the UNet backward ends -- graph 2 of the step),
  bucket 1 = [lo, ema_numel): the output blocks + `out` (20.07 M, final after the output-block
             backward -- graph 1),
  bucket 2 = [ema_numel, numel): the cond stage, Encoder4 (1.37 M, final when its autograd
             backward ends -- graph 3).
`HipTrainer` launches bucket 1's all-reduce on a side stream while the middle / input blocks'
backward runs, bucket 0's while Encoder4's backward runs, then bucket 2, then the optimizer.
When the arena layout does not allow the split (or ENCDIFF_DP_SPLIT=0) the UNet range is ONE
bucket (final when the UNet backward ends) and the exchange has two buckets.  Over RCCL the reduction is ReduceOp.AVG; gloo
(CPU tests) has no AVG, so SUM + a scale is used there.

Wire format: fp32 by default (the reference's DDP all-reduces fp32 gradients).  With
``grad_dtype=torch.bfloat16`` (ENCDIFF_DP_GRAD_BF16=1) each bucket is cast to a bf16 staging
buffer on the comm stream, all-reduced in bf16 (half the bytes over xGMI: 77.7 MB instead of
155.4 MB per step) and cast back into the fp32 arena before the optimizer; the ring's partial
sums are rounded to bf16 at every hop (~2^-9 relative per hop).

Collectives are issued by the host between graph replays, not captured: the host issues a
step's 4 replays + 3 all-reduces in well under 0.1 ms, far ahead of the ~10 ms of GPU work, so
capturing them would remove no GPU idle time (and could not be exercised on the one-GPU
boxes, where only gloo runs).

Bucket size: ``max_mb`` (ENCDIFF_DP_BUCKET_MB, bench.py --bucket-mb) cuts every coarse bucket
into all-reduces of at most that many MB of wire bytes (16-32 MB is SURVEY §8(e)'s range for
xGMI rings); the pieces of a coarse bucket are issued together, when its gradients are final.
0 keeps one all-reduce per coarse bucket.

Timing (``timing = True``): per step and coarse bucket, HIP events on the comm stream around
its all-reduces, so the exposed part of the exchange can be read on the first multi-GPU run
(``stats()``); the trainer adds the wait between the end of the backward and the optimizer.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def rank_seed(seed: int, rank: int) -> int:
    """Per-rank RNG stream (seed 1234 + rank)."""
    return seed + rank


def scaled_lr(base_lr: float, batch_per_gpu: int, world: int, accumulate: int = 1) -> float:
    """main_val.py:834-838: lr = accumulate_grad_batches * ngpu * batch_size * base_lr."""
    return accumulate * world * batch_per_gpu * base_lr


class GradBuckets:
    """Contiguous [lo, hi) element ranges of a flat gradient buffer, each all-reduced as
    one collective (mean over the process group)."""

    def __init__(self, flat: torch.Tensor, bounds: Sequence[int], group=None, grad_dtype=None,
                 max_mb: Optional[float] = None):
        assert flat.dim() == 1
        b = list(bounds)
        assert b[0] == 0 and b[-1] == flat.numel() and all(x < y for x, y in zip(b, b[1:])), b
        self.flat = flat
        self.bounds = b
        if max_mb is None:
            max_mb = float(os.environ.get("ENCDIFF_DP_BUCKET_MB", "0"))
        self.max_mb = max_mb
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # ENCDIFF_DP_FORCE=1 (one-rank process group): the collectives are issued anyway, so a
        # single-GPU box runs the exchange over RCCL exactly as an N-GPU node does
        self.active = self.world > 1 or (dist.is_initialized() and os.environ.get("ENCDIFF_DP_FORCE", "0") == "1")
        backend = dist.get_backend(group) if dist.is_initialized() else "none"
        self.native_avg = backend == "nccl"
        if grad_dtype is None:
            grad_dtype = torch.bfloat16 if os.environ.get("ENCDIFF_DP_GRAD_BF16", "0") == "1" else flat.dtype
        self.grad_dtype = grad_dtype
        # bf16 wire format: one staging buffer covering the whole arena (bucket views into it)
        self._wire = torch.empty(flat.numel(), dtype=grad_dtype, device=flat.device) \
            if grad_dtype != flat.dtype and self.active else None
        self.record = None  # tools/dp_check.py: {bucket: clone of what this rank sends}
        # pieces [lo, hi) of each coarse bucket, at most max_mb MB of wire bytes each (16-element aligned)
        esz = torch.tensor([], dtype=grad_dtype).element_size()
        cap = int(max_mb * 2 ** 20 / esz) // 16 * 16 if max_mb and max_mb > 0 else 0
        self.pieces = []
        for lo, hi in zip(b, b[1:]):
            n = max(1, -(-(hi - lo) // cap)) if cap else 1
            step = -(-(hi - lo) // n)
            step = -(-step // 16) * 16
            self.pieces.append([(x, min(hi, x + step)) for x in range(lo, hi, step)])
        self.timing = False
        self._events = []  # per step: {bucket: (start, done)} HIP events on the issuing stream

    @classmethod
    def from_arena(cls, arena, group=None, grad_dtype=None) -> "GradBuckets":
        bounds = [0]
        if 0 < arena.ema_numel < arena.numel:
            bounds.append(arena.ema_numel)
        bounds.append(arena.numel)
        return cls(arena.grad, bounds, group, grad_dtype)

    def __len__(self):
        return len(self.bounds) - 1

    def view(self, i: int) -> torch.Tensor:
        return self.flat[self.bounds[i]:self.bounds[i + 1]]

    def wire(self, i: int) -> torch.Tensor:
        """The buffer bucket i travels in (the gradient itself, or its bf16 staging view)."""
        if self._wire is None:
            return self.view(i)
        return self._wire[self.bounds[i]:self.bounds[i + 1]]

    def start(self, i: int, async_op: bool = True):
        """Launch bucket i's all-reduces (one per piece) in the calling stream's order; returns
        the works.  With timing on, HIP events bracket them on the calling stream."""
        if not self.active:
            return None
        op = dist.ReduceOp.AVG if self.native_avg else dist.ReduceOp.SUM
        if self.record is not None:
            self.record[i] = self.view(i).clone()
        if self._wire is not None:
            self.wire(i).copy_(self.view(i))  # fp32 -> bf16 on the calling (comm) stream
        ev0 = None
        if self.timing and torch.cuda.is_available() and self.flat.is_cuda:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        src = self._wire if self._wire is not None else self.flat
        works = [dist.all_reduce(src[lo:hi], op=op, group=self.group, async_op=async_op) for lo, hi in self.pieces[i]]
        if ev0 is not None:  # the issuing stream waits for the pieces: the done event marks their end
            for w in works:
                if w is not None:
                    w.wait()
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            if not self._events or i in self._events[-1]:
                self._events.append({})
            self._events[-1][i] = (ev0, ev1)
        return works

    def finish(self, i: int, works) -> None:
        """Wait for bucket i (the current stream waits on the collectives), cast back from the
        wire format and scale when the backend has no native average."""
        for w in works or ():
            if w is not None:
                w.wait()
        if self.active:
            if self._wire is not None:
                self.view(i).copy_(self.wire(i))
            if not self.native_avg:
                self.view(i).div_(self.world)

    def stats(self, clear: bool = True):
        """Mean milliseconds per step of each coarse bucket's all-reduces (timing on)."""
        torch.cuda.synchronize()
        acc = {}
        for st in self._events:
            for i, (e0, e1) in st.items():
                acc.setdefault(i, []).append(e0.elapsed_time(e1))
        if clear:
            self._events = []
        out = []
        for i in range(len(self)):
            v = acc.get(i, [])
            esz = self.wire(i).element_size()
            out.append({"bucket": i, "params": self.bounds[i + 1] - self.bounds[i],
                        "wire_mb": round((self.bounds[i + 1] - self.bounds[i]) * esz / 2 ** 20, 2),
                        "pieces": len(self.pieces[i]),
                        "allreduce_ms": round(sum(v) / len(v), 4) if v else None})
        return out

    def allreduce_all(self) -> None:
        works: List[Optional[object]] = [self.start(i) for i in range(len(self))]
        for i, w in enumerate(works):
            self.finish(i, w)
