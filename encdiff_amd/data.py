"""GPU-resident training images.

The reference streams Shapes3D through a DataLoader: uint8 HWC images
(disdata.py:45-97) -> ToTensor -> Normalize((0.5,)*3, (0.5,)*3) -> HWC float batch, then
get_input's 'b h w c -> b c h w' (ddpm_enc.py:347-353), 8 CPU workers and an H2D copy per
step.  Here the whole uint8 dataset lives in HBM (Shapes3D: 480 000 x 64 x 64 x 3 =
5.9 GB; MPI3D_toy 12.7 GB — both small against 288 GB), and ONE kernel
(`encdiff_gather_images_u8`) gathers a batch in shuffled-epoch order and writes the
normalised fp32 NCHW batch.  The epoch permutation and the step counter are device
tensors, so a captured training-step graph walks the epoch by itself; the host only
reshuffles at epoch boundaries (DataLoader(shuffle=True), drop_last as batch | N).
With data parallelism every rank draws the same permutation and takes the disjoint
strided shard perm[rank::world] (DistributedSampler semantics).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import ops


class ImagePool:
    def __init__(self, images_u8: torch.Tensor, batch: int, device, seed: int = 1234, rank: int = 0,
                 world: int = 1):
        assert images_u8.dtype == torch.uint8 and images_u8.dim() == 4, "expects uint8 [N, H, W, C]"
        self.device = torch.device(device)
        self.images = images_u8.to(self.device).contiguous()
        self.n = self.images.shape[0]
        self.batch = batch
        self.rank, self.world = rank, world
        self.steps_per_epoch = (self.n // world) // batch
        assert self.steps_per_epoch >= 1, "dataset smaller than one global batch"
        self.perm = torch.empty(self.steps_per_epoch * batch, dtype=torch.int64, device=self.device)
        self.step = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.gen = torch.Generator(device=self.device).manual_seed(seed)  # same on every rank
        self.epoch = -1
        self.host_step = 0
        self.reshuffle()

    # ------------------------------------------------------------ construction
    @classmethod
    def synthetic(cls, n: int, batch: int, device, h: int = 64, w: int = 64, c: int = 3, seed: int = 1234,
                  rank: int = 0, world: int = 1) -> "ImagePool":
        g = torch.Generator(device=device).manual_seed(seed)
        imgs = torch.randint(0, 256, (n, h, w, c), generator=g, device=device, dtype=torch.uint8)
        return cls(imgs, batch, device, seed, rank, world)

    @classmethod
    def from_npz(cls, path: str, batch: int, device, key: str = "images", **kw) -> "ImagePool":
        """Shapes3D npz layout of the reference loader (disdata.py:63-66); no pickle."""
        with np.load(path, allow_pickle=False) as d:
            imgs = torch.from_numpy(np.ascontiguousarray(d[key]))
        return cls(imgs, batch, device, **kw)

    # ------------------------------------------------------------ epoch order
    def reshuffle(self):
        full = torch.randperm(self.n, generator=self.gen, device=self.device)
        shard = full[self.rank::self.world][: self.perm.numel()]
        self.perm.copy_(shard)
        self.step.zero_()
        self.epoch += 1

    def draw(self, out: torch.Tensor, advance: bool = True):
        """Gather the next batch into out (fp32 [B, C, H, W]); stream-ordered, graph-safe.
        advance=False: peek (the device step counter stays, e.g. the scale_by_std batch)."""
        ops.gather_images_u8(self.images, self.perm, self.step, self.batch, out, advance=advance)

    def after_step(self):
        """Host bookkeeping once per step (outside graphs): new permutation per epoch."""
        self.host_step += 1
        if self.host_step % self.steps_per_epoch == 0:
            self.reshuffle()
