"""Data-parallel exchange of the EncDiff training step.

The step is pure data parallel: each rank draws its own batch and noise (seed 1234+rank),
runs the full step on its GPU, and the ONLY exchange is the mean of the gradients of the
38.84 M trainable parameters (UNet + Encoder4), which AdamW needs identical on every rank
(the reference gets the same from Lightning DDP, ddpm_enc.py:1598-1639 + main_val.py).

The gradient arena (`arena.ParamArena.grad`, one flat fp32 buffer) is split into
contiguous buckets in the order their gradients become final inside the step:
  bucket 0 = UNet parameters       (final when the UNet backward ends),
  bucket 1 = cond-stage parameters (final when Encoder4's autograd backward ends).
`HipTrainer` launches bucket 0's all-reduce on a side stream while Encoder4's backward
runs, then bucket 1, then the optimizer.  Over RCCL the reduction is ReduceOp.AVG; gloo
(CPU tests) has no AVG, so SUM + a scale is used there.

Wire format: fp32 by default (the reference's DDP all-reduces fp32 gradients).  With
``grad_dtype=torch.bfloat16`` (ENCDIFF_DP_GRAD_BF16=1) each bucket is cast to a bf16 staging
buffer on the comm stream, all-reduced in bf16 (half the bytes over xGMI: 77.7 MB instead of
155.4 MB per step) and cast back into the fp32 arena before the optimizer; the ring's partial
sums are rounded to bf16 at every hop (~2^-9 relative per hop).

Collectives are issued by the host between graph replays, not captured: the host issues a
step's 4 replays + 3 all-reduces in well under 0.1 ms, far ahead of the ~11 ms of GPU work, so
capturing them would remove no GPU idle time (and could not be exercised on the one-GPU
boxes, where only gloo runs).
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

    def __init__(self, flat: torch.Tensor, bounds: Sequence[int], group=None, grad_dtype=None):
        assert flat.dim() == 1
        b = list(bounds)
        assert b[0] == 0 and b[-1] == flat.numel() and all(x < y for x, y in zip(b, b[1:])), b
        self.flat = flat
        self.bounds = b
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        backend = dist.get_backend(group) if dist.is_initialized() else "none"
        self.native_avg = backend == "nccl"
        if grad_dtype is None:
            grad_dtype = torch.bfloat16 if os.environ.get("ENCDIFF_DP_GRAD_BF16", "0") == "1" else flat.dtype
        self.grad_dtype = grad_dtype
        # bf16 wire format: one staging buffer covering the whole arena (bucket views into it)
        self._wire = torch.empty(flat.numel(), dtype=grad_dtype, device=flat.device) \
            if grad_dtype != flat.dtype and self.world > 1 else None
        self.record = None  # tools/dp_check.py: {bucket: clone of what this rank sends}

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
        """Launch bucket i's all-reduce on the calling stream's order; returns the work."""
        if self.world == 1:
            return None
        op = dist.ReduceOp.AVG if self.native_avg else dist.ReduceOp.SUM
        w = self.wire(i)
        if self.record is not None:
            self.record[i] = self.view(i).clone()
        if self._wire is not None:
            w.copy_(self.view(i))  # fp32 -> bf16 on the calling (comm) stream
        return dist.all_reduce(w, op=op, group=self.group, async_op=async_op)

    def finish(self, i: int, work) -> None:
        """Wait for bucket i (the current stream waits on the collective), cast back from the
        wire format and scale when the backend has no native average."""
        if work is not None:
            work.wait()
        if self.world > 1:
            if self._wire is not None:
                self.view(i).copy_(self.wire(i))
            if not self.native_avg:
                self.view(i).div_(self.world)

    def allreduce_all(self) -> None:
        works: List[Optional[object]] = [self.start(i) for i in range(len(self))]
        for i, w in enumerate(works):
            self.finish(i, w)
