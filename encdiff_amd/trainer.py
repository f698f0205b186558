"""One EncDiff training step on the MI355X, captured as a HIP graph.

Step = (per rank)
  VQ encode (frozen, as-is) -> z * scale_factor
  Encoder4 (as-is, with grad) -> concept tokens c
  t ~ U{0..T-1}, eps ~ N(0, I), x_t = q_sample (HIP)
  eps_hat = UNet(x_t, t, c)          (HIP executor, forward)
  L1 loss + gradient seed            (HIP)
  backward: UNet (HIP) -> d c -> Encoder4 (torch autograd)
  [world > 1: RCCL all-reduce (mean) of the gradient arena in buckets (dp.py), each on a
   side stream as soon as its gradients are final: the output-block / out parameters while
   the rest of the UNet backward runs, the remaining UNet parameters while Encoder4's
   backward runs, then Encoder4's]
  AdamW + EMA over the flat arena, bf16 repack of GEMM weights   (HIP)

The device work of a step is replayed from captured graphs: one graph for the
single-GPU step; with DP four graphs sharing one memory pool -- (forward + UNet output-block
backward), (rest of the UNet backward), (Encoder4 backward), (optimizer) -- around the bucket
all-reduces.  Only the per-step scalars (lr, bias corrections,
EMA decay) cross the host->device boundary, through a pinned 8-float buffer.
Reference: ddpm_enc.py:360-375, 399-401, 1040-1053, 1183-1253, 1598-1639;
main_val.py:818-842 (lr = ngpu * batch * base_lr).
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from .data import ImagePool
from .dp import GradBuckets, rank_seed, scaled_lr, world_info


def _plain(obj):
    """A state dict with numpy scalars turned into Python numbers (LambdaLR keeps the schedule's
    numpy values in _last_lr): loadable with torch.load(weights_only=True)."""
    import numpy as np
    if isinstance(obj, dict):
        return {k: _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_plain(v) for v in obj)
    if isinstance(obj, np.generic):
        return obj.item()
    return obj


class HipTrainer:
    def __init__(self, ldm, batch_size: int, base_lr: Optional[float] = None, graph: bool = True,
                 data: Optional[ImagePool] = None, pool_size: int = 480000, seed: int = 1234,
                 bucket_mb: float = 0.0):
        self.ldm = ldm
        self.dev = ldm.device
        self.B = batch_size
        self.rank, self.world = world_info()
        # the DP exchange path (side-stream bucketed all-reduce, split backward, four graphs) runs
        # at world > 1, or with ENCDIFF_DP_FORCE=1 on a one-rank process group: a single-GPU box
        # then exercises the RCCL calls and the split capture exactly as an 8-GPU node does
        self.dp = self.world > 1 or (os.environ.get("ENCDIFF_DP_FORCE", "0") == "1" and dist.is_available()
                                     and dist.is_initialized())
        ldm.train()
        arena = ldm.setup_hip_training()
        self.arena = arena
        base = base_lr if base_lr is not None else 2.0e-6
        ldm.learning_rate = scaled_lr(base, batch_size, self.world)  # main_val.py:834-838 (scale_lr)
        opt = ldm.configure_optimizers()
        if isinstance(opt, tuple) or isinstance(opt, list):
            self.opt = opt[0][0]
            self.sched = opt[1][0]["scheduler"]
        else:
            self.opt, self.sched = opt, None
        self.bucket_mb = bucket_mb if bucket_mb else None  # None: ENCDIFF_DP_BUCKET_MB (0 = coarse buckets)
        self.buckets = GradBuckets.from_arena(arena)
        if self.bucket_mb is not None:
            self.buckets = GradBuckets(arena.grad, self.buckets.bounds, max_mb=self.bucket_mb)
        self.dp_timing = False  # HIP events around the exchange (dp_stats)
        self._dp_ev = []
        self._comm = torch.cuda.Stream() if self.dp else None
        # ENCDIFF_OPT_OVERLAP=1 (one GPU): the UNet's AdamW + EMA + repack (part 0) on a side stream
        # under the cond stage's backward (the UNet gradients are final once its backward returns).
        # Off: measured 9.47 -> 10.0 ms/step with it (same results) -- the bandwidth-bound optimizer
        # grid takes the CUs the cond stage's small latency-bound kernels wait for
        self._overlap = (not self.dp and hasattr(self.opt, "launch_part")
                         and os.environ.get("ENCDIFF_OPT_OVERLAP", "0") == "1")
        self._opt_s = torch.cuda.Stream() if self._overlap else None
        self._opt_in_fb = False  # the last _fwd_bwd launched the optimizer itself
        self.unet = ldm.model.diffusion_model
        # DP: split the UNet backward after the output blocks so their gradient bucket is
        # all-reduced while the middle / input blocks run (ENCDIFF_DP_SPLIT=0 disables)
        self._split_want = self.dp and os.environ.get("ENCDIFF_DP_SPLIT", "1") != "0"
        self._split_lo: Optional[int] = None
        self._split_checked = False
        self._g_rest = None
        # image resolution: the latent size times the first stage's downsampling (VQ-f4: x4)
        self.res = ldm.image_size * (2 ** getattr(ldm, "num_downs", 2))
        if data is None:  # synthetic uint8 images of the dataset's shape, resident in HBM
            data = ImagePool.synthetic(pool_size, batch_size, self.dev, h=self.res, w=self.res, seed=seed,
                                       rank=self.rank, world=self.world)
        self.data = data
        self.img = torch.empty(batch_size, 3, self.res, self.res, device=self.dev)
        self.loss_buf = torch.zeros(4, device=self.dev)
        # direct executor path (see _fwd_bwd): the EncDiff objective only
        self._direct = (ldm.parameterization == "eps" and ldm.loss_type == "l1" and not ldm.learn_logvar and
                        float(ldm.original_elbo_weight) == 0.0 and float(ldm.l_simple_weight) == 1.0 and
                        os.environ.get("ENCDIFF_TRAIN_DIRECT", "1") != "0")
        z_shape = (batch_size, ldm.channels, ldm.image_size, ldm.image_size)
        self._xt = torch.empty(z_shape, device=self.dev)
        self._seed = torch.empty(z_shape, device=self.dev)
        self.graph = graph
        self._feed = None  # test hook: batch, t and noise from static buffers (enable_feed)
        self._g_fb = None
        self._g_cond = None
        self._g_opt = None
        self._c = self._dc = None
        torch.manual_seed(rank_seed(seed, self.rank))
        from . import ops
        self._t = torch.empty(batch_size, dtype=torch.long, device=self.dev)
        self._noise = torch.empty(z_shape, device=self.dev)
        self._pro = ops.StepPrologue(self.dev, seed=rank_seed(seed, self.rank))
        self._pro.set_jobs([self.arena.grad])
        self._pro_final = False  # statistics slots registered after the first step
        self._melk = False       # SIGUSR1 (install_signal_handlers): checkpoint at the step boundary
        self._ckptdir = "."

    def _slots(self):
        """The UNet executor's statistics-slot registry (None before the executor exists)."""
        ex = getattr(self.unet, "_ex", None)
        return ex.stat_slots if ex is not None else None

    def _prologue_regions(self):
        """After the first step: the prologue also zeroes every producer-statistics slot the
        step's kernels added into (seen by ops.st_tail_fwd), so no fill runs inside the step."""
        from . import ops
        if self._pro_final:
            return
        regions = self._slots().register() if self._slots() is not None else []
        self._pro.set_jobs([self.arena.grad] + regions)
        self._pro_final = True

    # ---------------------------------------------------------------- test hook
    def enable_feed(self):
        """Parity-test hook (call before capture): the step reads its image batch, timesteps
        and noise from static buffers -- ``feed_img`` (B, 3, res, res) fp32, ``feed_t`` (B,)
        int64, ``feed_noise`` like z -- instead of the image pool and the RNG.  The captured
        graph reads them on every replay, so a checker writes a step's inputs and replays the
        same graph the benchmark times."""
        z_shape = (self.B, self.ldm.channels, self.ldm.image_size, self.ldm.image_size)
        self._feed = dict(img=torch.zeros(self.B, 3, self.res, self.res, device=self.dev),
                          t=torch.zeros(self.B, dtype=torch.long, device=self.dev),
                          noise=torch.zeros(z_shape, device=self.dev))
        return self._feed

    # ---------------------------------------------------------------- device work
    def _draw_batch(self, advance=True):
        if self._feed is not None:
            self.img.copy_(self._feed["img"])
        else:
            self.data.draw(self.img, advance=advance)

    def _fwd_bwd(self):
        """Everything up to the UNet backward.  The loss and the UNet run on the executor
        directly (LatentDiffusion.p_losses restated without autograd: q_sample with the
        scale_factor folded in, UNet forward, the fused L1 loss + gradient seed, UNet backward);
        only the as-is Encoder4 keeps torch autograd, seeded with d(context).  At world size 1
        Encoder4's backward runs inside this; with DP it is deferred (`_cond_bwd`) so the UNet
        gradient buckets can be all-reduced meanwhile.  Objectives outside the EncDiff one (eps,
        L1, fixed logvar, no ELBO term) take the reference-API p_losses + loss.backward() path."""
        ldm = self.ldm
        from . import ops
        # the batch gather reads the pool's epoch step; the prologue (ONE launch) then zeroes the
        # gradient arena and the statistics slots the step adds into, draws t and the noise
        # (Philox) and advances the epoch step and its own counter
        self._draw_batch(advance=False)
        if self._feed is not None:
            t, noise = self._feed["t"], self._feed["noise"]
            self._pro(timesteps=ldm.num_timesteps, data_step=self.data.step)
        else:
            t, noise = self._t, self._noise
            self._pro(t, noise, timesteps=ldm.num_timesteps, data_step=self.data.step)
        self.unet.executor().stat_slots.begin_step(self._pro_final)  # (the executor exists from here on)
        with torch.no_grad():
            z = ldm.encode_first_stage(self.img)  # frozen VQ (HIP); scale_factor applied in q_sample
        c = ldm.get_learned_conditioning(self.img)
        if not self._direct:
            return self._fwd_bwd_api(z, c, t, noise)
        ex = self.unet.executor()
        ex.infer = False
        self.arena.attach_grads()
        sf = ldm.scale_factor
        if not isinstance(sf, torch.Tensor):
            sf = self._sf_dev = torch.full((1,), float(sf), device=self.dev)
        from . import ops
        ops.q_sample(z, noise, t, ldm.sqrt_alphas_cumprod, ldm.sqrt_one_minus_alphas_cumprod, self._xt, x0_scale=sf)
        eps = ex.forward(self._xt, t, c.detach().reshape(self.B, -1).float())
        ops.l1_loss(eps, noise, t, ldm.lvlb_weights, self.loss_buf[:2], grad=self._seed)
        if not self.dp:
            dc = ex.backward(self._seed)
            if self._overlap:
                # the UNet's last deferred weight-gradient finalize must land before its AdamW
                ops.flush()
                cur = torch.cuda.current_stream()
                self._opt_s.wait_stream(cur)
                with torch.cuda.stream(self._opt_s):
                    self.opt.launch_part(0)
                c.backward(dc.view_as(c))
                self.opt.launch_part(1)
                cur.wait_stream(self._opt_s)
                self._opt_in_fb = True
                return
            c.backward(dc.view_as(c))
            return
        if not self._split_checked:
            self._plan_split(ex)
        # split: d(context) is the executor's buffer, complete after backward_rest()
        dc = ex.backward(self._seed, split=self._split_lo is not None)
        self._c, self._dc = c, dc.view_as(c)

    def _fwd_bwd_api(self, z, c, t, noise):
        """The reference-API form (LatentDiffusion.p_losses + autograd) for other objectives."""
        ldm = self.ldm
        z = ldm.get_first_stage_encoding(z)
        if not self.dp:
            loss, ld = ldm.p_losses(z, c, t, noise)
            loss.backward()
        else:
            c_det = c.detach().requires_grad_(True)
            loss, ld = ldm.p_losses(z, c_det, t, noise)
            ex = self.unet._ex
            if not self._split_checked:
                self._plan_split(ex)
            ex.split_requested = self._split_lo is not None
            loss.backward()
            ex.split_requested = False
            self._c, self._dc = c, (ex.d_ctx if self._split_lo is not None else c_det.grad)
        self.loss_buf[0].copy_(ld["train/loss_simple"])
        self.loss_buf[1].copy_(ld["train/loss_vlb"])

    def _plan_split(self, ex):
        """Bucket bounds [0, lo) remaining UNet, [lo, ema_numel) output blocks + out,
        [ema_numel, numel) cond stage -- when the arena layout allows the split."""
        self._split_checked = True
        if not self._split_want:
            return
        a = self.arena
        lo = ex.split_plan(list(dict(self.unet.named_parameters())))
        if lo is None or not 0 < lo < a.ema_numel < a.numel:
            return
        if any(lo <= o < a.ema_numel and not ex._early_final(n) for n, (o, _) in a.offsets.items()):
            return
        self._split_lo = lo
        rec = self.buckets.record
        self.buckets = GradBuckets(a.grad, [0, lo, a.ema_numel, a.numel], self.buckets.group,
                                   self.buckets.grad_dtype, max_mb=self.buckets.max_mb)
        self.buckets.record = rec

    def _unet_rest(self):
        self.unet._ex.backward_rest()

    def _cond_bwd(self):
        self._c.backward(self._dc)
        # drop the autograd graph: a graph kept alive across steps pins AccumulateGrad
        # nodes created on another stream, which breaks the next capture
        self._c = self._dc = None

    def _exchange(self, cond_bwd, unet_rest=None):
        """DP gradient mean.  Unsplit: bucket 0 (UNet) on the side stream overlapped with
        the cond stage backward, then bucket 1 (cond stage).  Split (`unet_rest` given):
        bucket 1 (output blocks + out) overlapped with the rest of the UNet backward, bucket 0
        (remaining UNet) with the cond stage backward, then bucket 2.  The current stream
        waits for all of them."""
        cur = torch.cuda.current_stream()
        self.buckets.timing = self.dp_timing
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if self.dp_timing else None
        if unet_rest is not None:
            self._comm.wait_stream(cur)
            with torch.cuda.stream(self._comm):
                w_out = self.buckets.start(1)
            unet_rest()
            self._comm.wait_stream(cur)
            with torch.cuda.stream(self._comm):
                w_unet = self.buckets.start(0)
            cond_bwd()
            if ev:
                ev[0].record()  # the backward is complete
            w_cond = self.buckets.start(2)
            self.buckets.finish(1, w_out)
            self.buckets.finish(0, w_unet)
            self.buckets.finish(2, w_cond)
        else:
            self._comm.wait_stream(cur)
            with torch.cuda.stream(self._comm):
                w0 = self.buckets.start(0)
            cond_bwd()
            if ev:
                ev[0].record()
            w1 = self.buckets.start(1) if len(self.buckets) > 1 else None
            self.buckets.finish(0, w0)
            if len(self.buckets) > 1:
                self.buckets.finish(1, w1)
        if ev:
            ev[1].record()  # every bucket is reduced: the optimizer may start
            self._dp_ev.append(ev)

    def dp_stats(self):
        """Exchange timing of the steps run with dp_timing on: the exposed wait from the end of
        the backward to the optimizer's start (ms per step), and each coarse bucket's all-reduce
        time (its pieces issued together, measured on the stream that issued them)."""
        if not self._dp_ev:
            return None
        torch.cuda.synchronize()
        exp = [a.elapsed_time(b) for a, b in self._dp_ev]
        self._dp_ev = []
        return {"exposed_ms": round(sum(exp) / len(exp), 4), "exposed_ms_max": round(max(exp), 4),
                "bucket_mb": self.buckets.max_mb, "buckets": self.buckets.stats(),
                "split_backward": self._split_lo is not None}

    # ---------------------------------------------------------------- setup
    def init_scale_factor(self):
        """scale_by_std on the first batch (ddpm_enc.py:586-608), computed on rank 0 and
        broadcast (the reference's @rank_zero_only re-registration never reaches other ranks).
        The batch is peeked (the pool's step counter does not advance), so the epoch still
        visits every batch once."""
        self._draw_batch(advance=False)
        self.ldm.init_scale_factor({"image": self.img.permute(0, 2, 3, 1)})
        if self.dp:
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
        from . import ops
        self._prologue_regions()
        # capture_error_mode "thread_local" (every capture in the package): under the default
        # "global" mode ANY thread's unsafe HIP call invalidates the capture, and with RCCL the
        # process-group watchdog thread polls the earlier all-reduces' events (hipEventQuery)
        # at arbitrary moments -- a one-rank RCCL run lost its step capture to that
        # (hipErrorStreamCaptureInvalidated, then the watchdog aborts the process)
        with torch.cuda.stream(s):
            try:
                with torch.cuda.graph(self._g_fb, stream=s, capture_error_mode="thread_local"):
                    self._opt_in_fb = False
                    self._fwd_bwd()
                    if not self.dp and not self._opt_in_fb:
                        self.opt.launch()
                if self.dp:
                    pool = self._g_fb.pool()
                    if self._split_lo is not None:
                        self._g_rest = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(self._g_rest, stream=s, pool=pool, capture_error_mode="thread_local"):
                            self._unet_rest()
                    self._g_cond = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self._g_cond, stream=s, pool=pool, capture_error_mode="thread_local"):
                        self._cond_bwd()
                    self._g_opt = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self._g_opt, stream=s, pool=pool, capture_error_mode="thread_local"):
                        self.opt.launch()
            finally:
                self._slots() is not None and self._slots().begin_step(False)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

    # ---------------------------------------------------------------- steps
    def step_eager(self):
        from . import ops
        self.opt.stage_hyper()
        self._opt_in_fb = False
        try:
            self._fwd_bwd()
            if self.dp:
                self._exchange(self._cond_bwd, self._unet_rest if self._split_lo is not None else None)
        finally:
            self._slots() is not None and self._slots().begin_step(False)
        if not self._opt_in_fb:
            self.opt.launch()
        self._post()
        self._prologue_regions()

    def step(self):
        if self._g_fb is None:
            return self.step_eager()
        self.opt.stage_hyper()
        # a replay skips the eager paths' weight-version checks: repack the bf16 weights if the
        # parameters were changed in place since the last step (e.g. after an EMA scope)
        self.ldm.refresh_hip_weights()
        self._g_fb.replay()
        if self.dp:
            self._exchange(self._g_cond.replay, self._g_rest.replay if self._g_rest is not None else None)
            self._g_opt.replay()
        self._post()

    def _post(self):
        self.data.after_step()
        if self.sched is not None:
            self.sched.step()
        self.ldm.global_step += 1
        if self._melk:  # SIGUSR1 arrived during the step: the checkpoint at its boundary
            self._melk = False
            if self.rank == 0:
                print("Summoning checkpoint.", flush=True)
                self.save_checkpoint(os.path.join(self._ckptdir, "last.ckpt"))

    def save_checkpoint(self, path: str, epoch: int = 0):
        """The training state as a Lightning-layout .ckpt (what ``trainer.save_checkpoint`` writes,
        main_val.py:845-851): 'state_dict' (the module parameters and LitEma buffers -- views of
        the arenas the graph-replayed optimizer updates, so the state after the last step, which
        ``init_from_ckpt`` reads), 'epoch', 'global_step', and for a resume (``load_checkpoint``)
        Lightning's 'optimizer_states' / 'lr_schedulers' keys plus 'encdiff_data':
          optimizer_states[0] = {'state': {'exp_avg', 'exp_avg_sq'} as flat fp32 arena copies (the
            AdamW moments of every trainable parameter, arena order), 'step': the AdamW step count,
            'param_groups': lr / betas / eps / weight_decay, 'arena_names': the arena's parameter
            order} -- the fused optimizer keeps its moments in the arena, not per parameter,
          lr_schedulers[0] = the LambdaLR state_dict,
          encdiff_data = the image pool's epoch permutation and step (the next batch drawn)."""
        torch.cuda.synchronize()
        sd = {k: v.detach().to("cpu", copy=True).contiguous() for k, v in self.ldm.state_dict().items()}
        a, o = self.arena, self.opt
        opt_state = {"state": {"exp_avg": a.exp_avg.detach().cpu().clone(),
                               "exp_avg_sq": a.exp_avg_sq.detach().cpu().clone()},
                     "step": int(o.step_count),
                     "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in o.param_groups],
                     "arena_names": list(a.names)}
        ck = {"state_dict": sd, "epoch": int(epoch), "global_step": int(self.ldm.global_step),
              "optimizer_states": [opt_state],
              "lr_schedulers": [_plain(self.sched.state_dict())] if self.sched is not None else [],
              "encdiff_data": {"perm": self.data.perm.detach().cpu().clone(),
                               "step": self.data.step.detach().cpu().clone(),
                               "host_step": int(self.data.host_step), "epoch": int(self.data.epoch)}}
        torch.save(_plain(ck), path)

    def load_checkpoint(self, path: str):
        """Resume from ``save_checkpoint``'s file (the reference's ``-r`` path restores the same
        training state through Lightning): parameters + EMA, AdamW moments and step count, the LR
        schedule position, global_step and the data position.  Captured graphs stay valid: every
        restore writes into the existing arena / pool buffers."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        missing, unexpected = self.ldm.load_state_dict(ck["state_dict"], strict=False)
        if missing or unexpected:
            raise RuntimeError(f"checkpoint does not match the model: missing {missing}, unexpected {unexpected}")
        self.arena.mark_dirty()
        os_ = ck["optimizer_states"][0]
        if list(os_["arena_names"]) != list(self.arena.names):
            raise RuntimeError("checkpoint arena layout differs from this model's")
        self.arena.exp_avg.copy_(os_["state"]["exp_avg"])
        self.arena.exp_avg_sq.copy_(os_["state"]["exp_avg_sq"])
        self.opt.step_count = int(os_["step"])
        for g, saved in zip(self.opt.param_groups, os_["param_groups"]):
            g.update(saved)
        if self.sched is not None and ck.get("lr_schedulers"):
            self.sched.load_state_dict(ck["lr_schedulers"][0])
        self.ldm.global_step = int(ck["global_step"])
        d = ck.get("encdiff_data")
        if d is not None:
            self.data.perm.copy_(d["perm"])
            self.data.step.copy_(d["step"])
            self.data.host_step, self.data.epoch = int(d["host_step"]), int(d["epoch"])
        # the bf16 GEMM weight copies follow the restored parameters
        self.unet.executor()
        if hasattr(self.ldm.cond_stage_model, "repack_hip"):
            self.ldm.cond_stage_model.repack_hip()
        torch.cuda.synchronize()

    def install_signal_handlers(self, ckptdir: str):
        """main_val.py:845-862: SIGUSR1 summons a checkpoint -- rank 0 writes ``ckptdir/last.ckpt``.
        The handler only raises a flag (the signal may land inside a graph replay); the step in
        progress finishes and its boundary saves.  (The reference's SIGUSR2 starts a pudb session
        on rank 0: an interactive debugger, not reproduced.)"""
        import signal
        self._ckptdir = ckptdir
        os.makedirs(ckptdir, exist_ok=True)

        def melk(*_):
            self._melk = True
        signal.signal(signal.SIGUSR1, melk)

    def loss(self):
        return float(self.loss_buf[0])

    def eps(self):
        """The denoiser output of the last step (the executor's buffer set of this batch size;
        a forward at another batch size in between, e.g. sampling, swaps the executor's set)."""
        ex = self.unet._ex
        ex.bind(self.B)
        return ex.eps


def time_steps(trainer: HipTrainer, steps: int, events=None) -> float:
    """Barrier + sync on both sides; returns the wall time of exactly `steps` steps.  events: an
    optional (start, end) pair of timing events recorded around the steps on this rank's stream
    (this rank's own GPU time, without the waits of the closing barrier)."""
    if trainer.world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if events is not None:
        events[0].record()
    for _ in range(steps):
        trainer.step()
    if events is not None:
        events[1].record()
    torch.cuda.synchronize()
    if trainer.world > 1:
        dist.barrier()
    return time.perf_counter() - t0
