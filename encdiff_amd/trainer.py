"""One EncDiff training step on the MI355X, captured as a HIP graph.

Step = (per rank)
  VQ encode (frozen, as-is) -> z * scale_factor
  Encoder4 (as-is, with grad) -> concept tokens c
  t ~ U{0..T-1}, eps ~ N(0, I), x_t = q_sample (HIP)
  eps_hat = UNet(x_t, t, c)          (HIP executor, forward)
  L1 loss + gradient seed            (HIP)
  backward: UNet (HIP) -> d c -> Encoder4 (torch autograd)
  [world > 1: RCCL all-reduce (mean) of the flat gradient arena]
  AdamW + EMA over the flat arena, bf16 repack of GEMM weights   (HIP)

The device work of a step is replayed from captured graphs: one graph for the
single-GPU step, or (forward+backward) and (optimizer) graphs around the
all-reduce when data-parallel.  Only the per-step scalars (lr, bias corrections,
EMA decay) cross the host->device boundary, through a pinned 8-float buffer.
Reference: ddpm_enc.py:360-375, 399-401, 1040-1053, 1183-1253, 1598-1639;
main_val.py:818-842 (lr = ngpu * batch * base_lr).
"""
from __future__ import annotations

import time
from typing import Optional

import torch
import torch.distributed as dist


class HipTrainer:
    def __init__(self, ldm, batch_size: int, base_lr: Optional[float] = None, graph: bool = True,
                 data_pool: Optional[torch.Tensor] = None, pool_size: int = 2048, seed: int = 1234,
                 bucket_mb: float = 0.0):
        self.ldm = ldm
        self.dev = ldm.device
        self.B = batch_size
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        ldm.train()
        arena = ldm.setup_hip_training()
        self.arena = arena
        base = base_lr if base_lr is not None else 2.0e-6
        ldm.learning_rate = self.world * batch_size * base  # main_val.py:834-838 (scale_lr)
        opt = ldm.configure_optimizers()
        if isinstance(opt, tuple) or isinstance(opt, list):
            self.opt = opt[0][0]
            self.sched = opt[1][0]["scheduler"]
        else:
            self.opt, self.sched = opt, None
        g = torch.Generator(device=self.dev).manual_seed(seed + self.rank)
        if data_pool is None:  # synthetic Shapes3D-shaped images in [-1, 1], resident in HBM
            data_pool = torch.rand(pool_size, 3, 64, 64, device=self.dev, generator=g) * 2 - 1
        self.pool = data_pool
        self.img = torch.empty(batch_size, 3, 64, 64, device=self.dev)
        self.loss_buf = torch.zeros(4, device=self.dev)
        self.graph = graph
        self._g_fb = None
        self._g_opt = None
        torch.manual_seed(seed + self.rank)

    # ---------------------------------------------------------------- device work
    def _draw_batch(self):
        idx = torch.randint(0, self.pool.shape[0], (self.B,), device=self.dev)
        torch.index_select(self.pool, 0, idx, out=self.img)

    def _fwd_bwd(self):
        ldm = self.ldm
        self.arena.grad.zero_()
        self._draw_batch()
        with torch.no_grad():
            z = ldm.get_first_stage_encoding(ldm.encode_first_stage(self.img)).detach()
        c = ldm.get_learned_conditioning(self.img)
        t = torch.randint(0, ldm.num_timesteps, (self.B,), device=self.dev)
        noise = torch.randn_like(z)
        loss, ld = ldm.p_losses(z, c, t, noise)
        loss.backward()
        self.loss_buf[0].copy_(ld["train/loss_simple"])
        self.loss_buf[1].copy_(ld["train/loss_vlb"])

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.arena.grad, op=dist.ReduceOp.AVG)

    # ---------------------------------------------------------------- setup
    def init_scale_factor(self):
        """scale_by_std on the first batch (ddpm_enc.py:586-608), computed on rank 0 and
        broadcast (the reference's @rank_zero_only re-registration never reaches other ranks)."""
        self._draw_batch()
        self.ldm.init_scale_factor({"image": self.img.permute(0, 2, 3, 1)})
        if self.world > 1:
            dist.broadcast(self.ldm.scale_factor, 0)

    def capture(self, warmup: int = 3):
        """Eager warm-up steps (allocations, MIOpen kernel selection, kernel attributes),
        then graph capture."""
        for _ in range(warmup):
            self.step_eager()
        torch.cuda.synchronize()
        if not self.graph:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        self._g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(self._g_fb, stream=s):
                self._fwd_bwd()
                if self.world == 1:
                    self.opt.launch()
            if self.world > 1:
                self._g_opt = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._g_opt, stream=s):
                    self.opt.launch()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

    # ---------------------------------------------------------------- steps
    def step_eager(self):
        self.opt.stage_hyper()
        self._fwd_bwd()
        self._allreduce()
        self.opt.launch()
        self._post()

    def step(self):
        if self._g_fb is None:
            return self.step_eager()
        self.opt.stage_hyper()
        self._g_fb.replay()
        if self.world > 1:
            self._allreduce()
            self._g_opt.replay()
        self._post()

    def _post(self):
        if self.sched is not None:
            self.sched.step()
        self.ldm.global_step += 1

    def loss(self):
        return float(self.loss_buf[0])


def time_steps(trainer: HipTrainer, steps: int) -> float:
    """Barrier + sync on both sides; returns the wall time of exactly `steps` steps."""
    if trainer.world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        trainer.step()
    torch.cuda.synchronize()
    if trainer.world > 1:
        dist.barrier()
    return time.perf_counter() - t0
