"""Data-parallel exchange (encdiff_amd/dp.py) on CPU: world size 2 over gloo.

Covers the DP contract of SURVEY.md §8(e): per-rank seeds, lr scaling, the two-bucket
gradient mean (UNet | cond stage) equal to a full-buffer mean, data-parallel gradients
equal to the single-process full-batch gradient, identical optimizer steps on every rank,
and the rank-0 broadcast of scale_factor.
"""
from __future__ import annotations

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from encdiff_amd import dp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeArena:
    def __init__(self, numel, ema_numel):
        self.numel, self.ema_numel = numel, ema_numel
        self.grad = torch.zeros(numel)


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, w = dp.world_info()
        assert (r, w) == (rank, world)
        res = {}
        # 1. bucketed mean == full mean
        ar = _FakeArena(1000, 640)
        g = torch.Generator().manual_seed(dp.rank_seed(1234, rank))
        ar.grad.copy_(torch.randn(1000, generator=g))
        full = ar.grad.clone()
        dist.all_reduce(full)
        full /= world
        b = dp.GradBuckets.from_arena(ar)
        assert len(b) == 2 and b.bounds == [0, 640, 1000]
        w0 = b.start(0)
        w1 = b.start(1)
        b.finish(0, w0)
        b.finish(1, w1)
        res["bucket_err"] = float((ar.grad - full).abs().max())
        # 1a. the bucket-size knob: each coarse bucket cut into pieces of <= max_mb, same mean
        ar.grad.copy_(torch.randn(1000, generator=torch.Generator().manual_seed(dp.rank_seed(7, rank))))
        full = ar.grad.clone()
        dist.all_reduce(full)
        full /= world
        bp = dp.GradBuckets.from_arena(ar)
        bp = dp.GradBuckets(ar.grad, bp.bounds, max_mb=256 * 4 / 2 ** 20)  # 256 fp32 per piece
        assert [len(p) for p in bp.pieces] == [3, 2] and bp.pieces[0][0] == (0, 224)
        assert all(hi - lo <= 256 for pc in bp.pieces for lo, hi in pc)
        assert [pc[0][0] for pc in bp.pieces] == [0, 640] and [pc[-1][1] for pc in bp.pieces] == [640, 1000]
        bp.allreduce_all()
        res["piece_err"] = float((ar.grad - full).abs().max())
        # 1b. the same in the bf16 wire format: mean within bf16 rounding, equal on all ranks
        ar.grad.copy_(torch.randn(1000, generator=torch.Generator().manual_seed(dp.rank_seed(99, rank))))
        full = ar.grad.clone()
        dist.all_reduce(full)
        full /= world
        b16 = dp.GradBuckets.from_arena(ar, grad_dtype=torch.bfloat16)
        assert b16.wire(0).dtype == torch.bfloat16 and ar.grad.dtype == torch.float32
        b16.allreduce_all()
        res["bf16_rel"] = float((ar.grad - full).norm() / full.norm())
        res["bf16_vals"] = ar.grad.clone()
        # 2. DP gradient of a mean loss over per-rank halves == full-batch gradient
        torch.manual_seed(0)
        lin = torch.nn.Linear(16, 8)
        X = torch.randn(8, 16)
        Y = torch.randn(8, 8)
        xs, ys = X[rank * 4:(rank + 1) * 4], Y[rank * 4:(rank + 1) * 4]
        (lin(xs) - ys).abs().mean().backward()
        flat = torch.cat([p.grad.reshape(-1) for p in lin.parameters()])
        gb = dp.GradBuckets(flat, [0, 8 * 16, flat.numel()])
        gb.allreduce_all()
        lin.zero_grad()
        (lin(X) - Y).abs().mean().backward()
        ref = torch.cat([p.grad.reshape(-1) for p in lin.parameters()])
        res["dp_grad_err"] = float((flat - ref).abs().max())
        # 3. identical AdamW step on every rank after the exchange
        p = torch.cat([q.detach().reshape(-1) for q in lin.parameters()])
        opt_p = torch.nn.Parameter(p.clone())
        opt_p.grad = flat.clone()
        opt = torch.optim.AdamW([opt_p], lr=dp.scaled_lr(2e-6, 128, world))
        opt.step()
        gathered = [torch.empty_like(opt_p.data) for _ in range(world)]
        dist.all_gather(gathered, opt_p.data)
        res["opt_rank_diff"] = float((gathered[0] - gathered[1]).abs().max())
        # 4. scale_factor broadcast from rank 0
        sf = torch.tensor([0.5 + rank])
        dist.broadcast(sf, 0)
        res["scale_factor"] = float(sf)
        torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_seed_and_lr():
    assert dp.rank_seed(1234, 3) == 1237
    assert dp.scaled_lr(2e-6, 128, 8) == pytest.approx(2.048e-3)
    assert dp.scaled_lr(2e-6, 4, 1) == pytest.approx(8e-6)


def test_buckets_single_process():
    ar = _FakeArena(100, 60)
    ar.grad.normal_()
    before = ar.grad.clone()
    b = dp.GradBuckets.from_arena(ar)
    b.allreduce_all()  # world 1: no-op
    assert torch.equal(before, ar.grad)
    assert torch.equal(b.view(1), ar.grad[60:])


def test_gloo_world2():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world, start_method="spawn", join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert torch.equal(res[0]["bf16_vals"], res[1]["bf16_vals"])
    for r in res:
        assert r["bf16_rel"] < 1e-2
        assert r["bucket_err"] < 1e-6
        assert r["piece_err"] < 1e-6
        assert r["dp_grad_err"] < 1e-6
        assert r["opt_rank_diff"] == 0.0
        assert r["scale_factor"] == 0.5


def test_image_pool_shards():
    """DistributedSampler semantics of the HBM dataset: same permutation on every rank,
    disjoint strided shards, new permutation per epoch (host side, CPU tensors)."""
    from encdiff_amd.data import ImagePool
    imgs = torch.zeros(103, 4, 4, 3, dtype=torch.uint8)
    p0 = ImagePool(imgs, 8, "cpu", seed=5, rank=0, world=2)
    p1 = ImagePool(imgs, 8, "cpu", seed=5, rank=1, world=2)
    assert p0.steps_per_epoch == 6 and p0.perm.numel() == 48
    a, b = set(p0.perm.tolist()), set(p1.perm.tolist())
    assert not (a & b) and a | b <= set(range(103))
    first = p0.perm.clone()
    for _ in range(p0.steps_per_epoch):
        p0.after_step()
    assert p0.epoch == 1 and not torch.equal(first, p0.perm)
