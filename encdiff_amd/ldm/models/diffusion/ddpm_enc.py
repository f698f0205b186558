"""DDPM / LatentDiffusion / DiffusionWrapper -- mirror of
ldm/models/diffusion/ddpm_enc.py for the EncDiff denoising path.

Same constructor kwargs (configs/latent-diffusion/*.yaml load unchanged), same
buffer / submodule names (state_dict keys identical to the reference: model.*,
model_ema.*, first_stage_model.*, cond_stage_model.*, the schedule buffers and
scale_factor), same methods on the path: register_schedule (:133-187),
q_sample (:292-295), get_input (:773-844), forward (:1040-1053),
apply_model (:1065-1163), p_losses (:1183-1253), training_step (:360-375),
on_train_batch_end / EMA (:399-401), configure_optimizers (:1598-1639),
sample_log (:1442-1455), log_images (:1473-1596, sampling subset).

The modules are plain nn.Modules (no Lightning dependency); ``training_step`` returns
the loss and keeps the reference's log dict in ``self.last_log``.  q_sample, the UNet,
the L1 loss and its gradient seed run on the HIP path; the frozen VQ encoder and the
concept encoder Encoder4 are called as-is.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from functools import partial

import numpy as np
import torch
from torch import nn

from encdiff_amd import ops, torch_ops  # noqa: F401  (torch_ops registers torch.ops.encdiff.*)
from ...util import count_params, default, exists, instantiate_from_config
from ...modules.diffusionmodules.util import extract_into_tensor, make_beta_schedule
from ...modules.ema import LitEma
from ..autoencoder import IdentityFirstStage, VQModelInterface
from .ddim import DDIMSampler

__conditioning_keys__ = {"concat": "c_concat", "crossattn": "c_crossattn", "adm": "y"}


def disabled_train(self, mode=True):
    return self


class _PLossFn(torch.autograd.Function):
    """L1 eps-prediction loss of p_losses (ddpm_enc.py:1194-1213) on the HIP path:
    forward -> (loss, loss_vlb) and the gradient seed sign(pred - eps)/(B*CHW) in one
    kernel; backward scales the seed by the incoming gradient."""

    @staticmethod
    def forward(ctx, pred, noise, t, lvlb, l_simple_weight):
        out2, seed = torch.ops.encdiff.l1_loss(pred, noise, t, lvlb, float(l_simple_weight))
        ctx.save_for_backward(seed)
        ctx.mark_non_differentiable(out2)
        return out2[0].clone(), out2[1].clone()

    @staticmethod
    def backward(ctx, g_loss, g_vlb):
        (seed,) = ctx.saved_tensors
        return seed * g_loss, None, None, None, None


class FusedArenaAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics (defaults of ddpm_enc.py:1615) as ONE HIP kernel over
    the parameter arena, with the LitEma update fused in and the bf16 GEMM weights
    repacked right after.  Compatible with torch LambdaLR (param_groups[0]['lr'])."""

    def __init__(self, params, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, ema=None,
                 repack=None, repack_parts=None):
        super().__init__(list(params), dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.arena = arena
        self.ema = ema
        self.repack = repack
        self.repack_parts = repack_parts  # (UNet repack, cond-stage repack) for launch_part
        self.step_count = 0
        # ring of pinned staging rows: a row is rewritten only after the H2D copy that read it
        # has run (its event), so a host running steps ahead of the GPU never changes the
        # scalars of a step still queued
        ring = int(os.environ.get("ENCDIFF_HYPER_RING", "32"))
        self._host = torch.zeros(max(ring, 1), 8, dtype=torch.float32).pin_memory() if torch.cuda.is_available() else None
        self._host_ev = [None] * ring
        self._host_i = 0

    def hyper_values(self):
        g = self.param_groups[0]
        omd = self.ema.next_decay() if self.ema is not None else 0.0
        return ops.adamw_hyper(g["lr"], self.step_count, g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"],
                               omd)

    def stage_hyper(self):
        """Host -> device copy of this step's scalars (outside any captured graph)."""
        self.step_count += 1
        self._opt_called = True  # tells torch LR schedulers the optimizer stepped (launch() bypasses step())
        vals = self.hyper_values()
        if self._host is not None:
            if not self._host_ev:  # ENCDIFF_HYPER_RING=0: one unguarded row (A/B only)
                self._host[0].copy_(torch.tensor(vals, dtype=torch.float32))
                self.arena.hyper.copy_(self._host[0], non_blocking=True)
                return
            i = self._host_i
            self._host_i = (i + 1) % len(self._host_ev)
            if self._host_ev[i] is not None:
                self._host_ev[i].synchronize()
            row = self._host[i]
            row.copy_(torch.tensor(vals, dtype=torch.float32))
            self.arena.hyper.copy_(row, non_blocking=True)
            ev = self._host_ev[i] = self._host_ev[i] or torch.cuda.Event()
            ev.record()
        else:
            self.arena.hyper.copy_(torch.tensor(vals, dtype=torch.float32))

    def launch(self):
        """Device work of one step (capturable): AdamW + EMA, then bf16 repack."""
        a = self.arena
        ema = a.ema if self.ema is not None else None
        ops.adamw_ema(a.master, a.grad, a.exp_avg, a.exp_avg_sq, a.hyper, ema=ema,
                      ema_n=a.ema_numel if ema is not None else 0, mirror=a.mirror)
        if self.repack is not None:
            a.mirror_fresh = a.mirror is not None  # the update wrote the bf16 mirror: packs skip it
            try:
                self.repack()
            finally:
                a.mirror_fresh = False

    def launch_part(self, part: int):
        """The same update in two launches over the arena's two ranges: part 0 = [0, ema_numel)
        (the UNet, with the EMA) + the UNet's bf16 repack, part 1 = the rest (the cond stage) + its
        repack.  The trainer runs part 0 on a side stream while the cond stage's backward runs
        (the UNet gradients are final by then); element-wise, so the result is the one launch's."""
        a = self.arena
        mid = (a.ema_numel + 3) // 4 * 4  # float4 lanes: the split on a 4-element boundary (the
        # elements up to it past ema_numel are the next parameter's alignment padding)
        lo, hi = (0, mid) if part == 0 else (mid, a.numel)
        if hi > lo:
            ema = a.ema if (self.ema is not None and part == 0) else None
            ops.adamw_ema(a.master[lo:hi], a.grad[lo:hi], a.exp_avg[lo:hi], a.exp_avg_sq[lo:hi], a.hyper, ema=ema,
                          ema_n=a.ema_numel if ema is not None else 0,
                          mirror=a.mirror[lo:hi] if a.mirror is not None else None)
        if self.repack_parts is not None:
            a.mirror_fresh = a.mirror is not None and hi > lo
            try:
                self.repack_parts[part]()
            finally:
                a.mirror_fresh = False

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.stage_hyper()
        self.launch()
        return loss

    def zero_grad(self, set_to_none: bool = True):
        """Lightning calls this every step.  torch's default walks ~1900 parameters (and with
        set_to_none the next backward re-attaches each arena view with a zero launch of its own);
        here the parameters keep their arena views and the whole gradient arena is zeroed in ONE
        launch -- .grad reads as zeros, not None, whichever flag is passed."""
        self.arena.zero_grad()


class DDPM(nn.Module):
    """ddpm_enc.py:48-479 (the parts on the EncDiff path)."""

    def __init__(self, unet_config, timesteps=1000, beta_schedule="linear", loss_type="l2", ckpt_path=None,
                 ignore_keys=[], load_only_unet=False, monitor="val/loss", use_ema=True, first_stage_key="image",
                 image_size=256, channels=3, log_every_t=100, clip_denoised=True, linear_start=1e-4,
                 linear_end=2e-2, cosine_s=8e-3, given_betas=None, original_elbo_weight=0., v_posterior=0.,
                 l_simple_weight=1., conditioning_key=None, parameterization="eps", scheduler_config=None,
                 use_positional_encodings=False, learn_logvar=False, logvar_init=0., eval_name=None):
        super().__init__()
        assert parameterization in ["eps", "x0"]
        self.parameterization = parameterization
        self.cond_stage_model = None
        self.clip_denoised = clip_denoised
        self.log_every_t = log_every_t
        self.first_stage_key = first_stage_key
        self.image_size = image_size
        self.channels = channels
        self.use_positional_encodings = use_positional_encodings
        self.model = DiffusionWrapper(unet_config, conditioning_key)
        count_params(self.model, verbose=True)
        self.use_ema = use_ema
        if self.use_ema:
            self.model_ema = LitEma(self.model)
        self.use_scheduler = scheduler_config is not None
        if self.use_scheduler:
            self.scheduler_config = scheduler_config
        self.v_posterior = v_posterior
        self.original_elbo_weight = original_elbo_weight
        self.l_simple_weight = l_simple_weight
        if monitor is not None:
            self.monitor = monitor
        self.eval_name = eval_name  # disentanglement metrics are out of scope
        if ckpt_path is not None:
            self.init_from_ckpt(ckpt_path, ignore_keys=ignore_keys, only_model=load_only_unet)
        self.register_schedule(given_betas=given_betas, beta_schedule=beta_schedule, timesteps=timesteps,
                               linear_start=linear_start, linear_end=linear_end, cosine_s=cosine_s)
        self.loss_type = loss_type
        self.learn_logvar = learn_logvar
        self.logvar = torch.full(fill_value=logvar_init, size=(self.num_timesteps,))
        if self.learn_logvar:
            self.logvar = nn.Parameter(self.logvar, requires_grad=True)
        self.global_step = 0
        self.current_epoch = 0
        self.last_log = {}

    @property
    def device(self):
        return self.betas.device

    def register_schedule(self, given_betas=None, beta_schedule="linear", timesteps=1000, linear_start=1e-4,
                          linear_end=2e-2, cosine_s=8e-3):
        """ddpm_enc.py:133-187."""
        betas = given_betas if exists(given_betas) else make_beta_schedule(
            beta_schedule, timesteps, linear_start=linear_start, linear_end=linear_end, cosine_s=cosine_s)
        alphas = 1. - betas
        ac = np.cumprod(alphas, axis=0)
        ac_prev = np.append(1., ac[:-1])
        ac_next = np.append(ac[1:], ac[-1])
        self.num_timesteps = int(betas.shape[0])
        self.linear_start, self.linear_end = linear_start, linear_end
        to_torch = partial(torch.tensor, dtype=torch.float32)
        self.register_buffer("betas", to_torch(betas))
        self.register_buffer("alphas_cumprod", to_torch(ac))
        self.register_buffer("alphas_cumprod_prev", to_torch(ac_prev))
        self.register_buffer("alphas_cumprod_next", to_torch(ac_next))
        self.register_buffer("sqrt_alphas_cumprod", to_torch(np.sqrt(ac)))
        self.register_buffer("sqrt_one_minus_alphas_cumprod", to_torch(np.sqrt(1. - ac)))
        self.register_buffer("log_one_minus_alphas_cumprod", to_torch(np.log(1. - ac)))
        self.register_buffer("sqrt_recip_alphas_cumprod", to_torch(np.sqrt(1. / ac)))
        self.register_buffer("sqrt_recipm1_alphas_cumprod", to_torch(np.sqrt(1. / ac - 1)))
        pv = (1 - self.v_posterior) * betas * (1. - ac_prev) / (1. - ac) + self.v_posterior * betas
        self.register_buffer("posterior_variance", to_torch(pv))
        self.register_buffer("posterior_log_variance_clipped", to_torch(np.log(np.maximum(pv, 1e-20))))
        self.register_buffer("posterior_mean_coef1", to_torch(betas * np.sqrt(ac_prev) / (1. - ac)))
        self.register_buffer("posterior_mean_coef2", to_torch((1. - ac_prev) * np.sqrt(alphas) / (1. - ac)))
        if self.parameterization == "eps":
            lv = self.betas ** 2 / (2 * self.posterior_variance * to_torch(alphas) * (1 - self.alphas_cumprod))
        else:
            lv = 0.5 * np.sqrt(torch.Tensor(ac)) / (2. * 1 - torch.Tensor(ac))
        lv[0] = lv[1]
        self.register_buffer("lvlb_weights", lv, persistent=False)

    @contextmanager
    def ema_scope(self, context=None):
        """ddpm_enc.py:189-202."""
        if self.use_ema:
            self.model_ema.store(self.model.parameters())
            self.model_ema.copy_to(self.model)
            self._weights_changed()
        try:
            yield None
        finally:
            if self.use_ema:
                self.model_ema.restore(self.model.parameters())
                self._weights_changed()

    def refresh_hip_weights(self):
        """Bring the bf16 weight packs up to date with the fp32 parameters before a captured
        graph is replayed: a replay skips UNetModel.executor() / Encoder4._encode, where the
        eager path checks for in-place parameter changes (EMA swap, load_state_dict, arena
        writes).  Host-side version checks; a repack launch only when something changed."""
        unet = self.model.diffusion_model
        if getattr(unet, "_arena", None) is not None:
            unet.executor()
        cs = self.cond_stage_model
        tr = getattr(cs, "_trunk", None)
        if tr is not None and (tr.arena.master._version, tr.arena.gen) != cs._trunk_version:
            cs.repack_hip()

    def _weights_changed(self):
        """Parameters were rewritten through their .data views (EMA swap): the UNet's bf16
        weight packs must be refreshed before the next forward."""
        a = getattr(self.model.diffusion_model, "_arena", None)
        if a is not None:
            a.mark_dirty()

    def init_from_ckpt(self, path, ignore_keys=list(), only_model=False):
        """ddpm_enc.py:204-220 (weights-only load; strict=False)."""
        sd = torch.load(path, map_location="cpu", weights_only=True)
        sd = sd.get("state_dict", sd)
        for k in list(sd.keys()):
            if any(k.startswith(ik) for ik in ignore_keys):
                del sd[k]
        target = self.model if only_model else self
        missing, unexpected = target.load_state_dict(sd, strict=False)
        print(f"Restored from {path} with {len(missing)} missing and {len(unexpected)} unexpected keys")
        return missing, unexpected

    def q_sample(self, x_start, t, noise=None):
        """ddpm_enc.py:292-295 -- one HIP kernel."""
        noise = default(noise, lambda: torch.randn_like(x_start))
        if not x_start.is_cuda:
            raise RuntimeError("q_sample runs on the HIP path")
        return torch.ops.encdiff.q_sample(x_start, noise, t, self.sqrt_alphas_cumprod,
                                          self.sqrt_one_minus_alphas_cumprod)

    def get_loss(self, pred, target, mean=True):
        if self.loss_type == "l1":
            loss = (target - pred).abs()
            return loss.mean() if mean else loss
        if self.loss_type == "l2":
            return torch.nn.functional.mse_loss(target, pred, reduction="mean" if mean else "none")
        raise NotImplementedError(self.loss_type)

    def get_input(self, batch, k):
        """ddpm_enc.py:347-353: HWC batch -> NCHW float."""
        x = batch[k]
        if len(x.shape) == 3:
            x = x[..., None]
        return x.permute(0, 3, 1, 2).contiguous(memory_format=torch.contiguous_format).float()

    def training_step(self, batch, batch_idx=0):
        loss, loss_dict = self.shared_step(batch)
        self.last_log = dict(loss_dict)
        self.last_log["global_step"] = self.global_step
        return loss

    def on_train_batch_end(self, *args, **kwargs):
        """ddpm_enc.py:399-401 (skipped when the EMA is fused into the optimizer kernel)."""
        if self.use_ema and not getattr(self, "_ema_fused", False):
            self.model_ema(self.model)
        self.global_step += 1


class LatentDiffusion(DDPM):
    """ddpm_enc.py:482-1648 (EncDiff path)."""

    def __init__(self, first_stage_config, cond_stage_config, num_timesteps_cond=None, cond_stage_key="image",
                 cond_stage_trainable=False, concat_mode=True, cond_stage_forward=None, conditioning_key=None,
                 scale_factor=1.0, scale_by_std=False, lambda_mcl=0.0, mcl_tau=0.1, mcl_proj_dim=128,
                 mcl_sigma=0.1, mcl_neg_mode="shuffle_u", mcl_type="infonce_mechgrad", use_mcl=False, *args,
                 **kwargs):
        self.num_timesteps_cond = default(num_timesteps_cond, 1)
        self.scale_by_std = scale_by_std
        assert self.num_timesteps_cond <= kwargs["timesteps"]
        if conditioning_key is None:
            conditioning_key = "concat" if concat_mode else "crossattn"
        if cond_stage_config == "__is_unconditional__":
            conditioning_key = None
        ckpt_path = kwargs.pop("ckpt_path", None)
        ignore_keys = kwargs.pop("ignore_keys", [])
        super().__init__(conditioning_key=conditioning_key, *args, **kwargs)
        if use_mcl and lambda_mcl > 0:
            raise NotImplementedError("MCL auxiliary losses are outside the HIP path scope (SURVEY.md §2 row 10)")
        self.concat_mode = concat_mode
        self.cond_stage_trainable = cond_stage_trainable
        self.cond_stage_key = cond_stage_key
        try:
            self.num_downs = len(first_stage_config["params"]["ddconfig"]["ch_mult"]) - 1
        except Exception:
            self.num_downs = 0
        if not scale_by_std:
            self.scale_factor = scale_factor
        else:
            self.register_buffer("scale_factor", torch.tensor(scale_factor))
        self.instantiate_first_stage(first_stage_config)
        self.instantiate_cond_stage(cond_stage_config)
        self.cond_stage_forward = cond_stage_forward
        self.clip_denoised = False
        self.restarted_from_ckpt = False
        self.shorten_cond_schedule = self.num_timesteps_cond > 1
        if self.shorten_cond_schedule:
            raise NotImplementedError("num_timesteps_cond > 1 is not used by EncDiff configs")
        if ckpt_path is not None:
            self.init_from_ckpt(ckpt_path, ignore_keys)
            self.restarted_from_ckpt = True
        self.use_mcl, self.lambda_mcl = use_mcl, lambda_mcl
        self._optimizer = None

    # ------------------------------------------------------------ stages
    def instantiate_first_stage(self, config):
        model = instantiate_from_config(config)
        if model is not None:
            self.first_stage_model = model.eval()
            self.first_stage_model.train = disabled_train.__get__(self.first_stage_model)
            for p in self.first_stage_model.parameters():
                p.requires_grad = False
        else:
            self.first_stage_model = None

    def instantiate_cond_stage(self, config):
        if not self.cond_stage_trainable:
            if config == "__is_first_stage__":
                self.cond_stage_model = self.first_stage_model
            elif config == "__is_unconditional__":
                self.cond_stage_model = None
            else:
                model = instantiate_from_config(config)
                self.cond_stage_model = model.eval()
                self.cond_stage_model.train = disabled_train.__get__(self.cond_stage_model)
                for p in self.cond_stage_model.parameters():
                    p.requires_grad = False
        else:
            self.cond_stage_model = instantiate_from_config(config)

    @torch.no_grad()
    def init_scale_factor(self, batch):
        """on_train_batch_start (ddpm_enc.py:586-608): scale_factor = 1/std(z) of the first batch."""
        if self.scale_by_std and self.global_step == 0 and not self.restarted_from_ckpt:
            x = DDPM.get_input(self, batch, self.first_stage_key).to(self.device)
            z = self.encode_first_stage(x).detach()
            self.scale_factor.copy_(1. / z.flatten().float().std())
        return self.scale_factor

    def get_first_stage_encoding(self, encoder_posterior):
        return self.scale_factor * encoder_posterior

    def get_learned_conditioning(self, c):
        if self.cond_stage_forward is None:
            if hasattr(self.cond_stage_model, "encode") and callable(self.cond_stage_model.encode):
                return self.cond_stage_model.encode(c)
            return self.cond_stage_model(c)
        return getattr(self.cond_stage_model, self.cond_stage_forward)(c)

    @torch.no_grad()
    def encode_first_stage(self, x):
        return x if self.first_stage_model is None else self.first_stage_model.encode(x)

    @torch.no_grad()
    def decode_first_stage(self, z, predict_cids=False, force_not_quantize=False, disentangled_repr=None):
        z = 1. / self.scale_factor * z
        if self.first_stage_model is None:
            return z
        if isinstance(self.first_stage_model, VQModelInterface):
            return self.first_stage_model.decode(z, force_not_quantize=predict_cids or force_not_quantize,
                                                 disentangled_repr=disentangled_repr)
        return self.first_stage_model.decode(z)

    @torch.no_grad()
    def get_input(self, batch, k, return_first_stage_outputs=False, force_c_encode=False, cond_key=None,
                  return_original_cond=False, bs=None, return_false=False, return_disentangled=False):
        """ddpm_enc.py:773-844 (cross-attention conditioning on the raw image)."""
        x = DDPM.get_input(self, batch, k)
        if bs is not None:
            x = x[:bs]
        x = x.to(self.device)
        z = self.get_first_stage_encoding(self.encode_first_stage(x)).detach()
        cond_key = cond_key or self.cond_stage_key
        xc = x if cond_key == self.first_stage_key else DDPM.get_input(self, batch, cond_key).to(self.device)
        cb = None
        if not self.cond_stage_trainable or force_c_encode:
            c = self.get_learned_conditioning(xc)
            if return_false:
                cb = self.cond_stage_model.encoding(xc)
        else:
            c = xc
        if bs is not None:
            c = c[:bs]
        out = [z, c]
        if return_first_stage_outputs:
            out.extend([x, self.decode_first_stage(z)])
        if return_original_cond:
            out.append(xc)
        if return_false:
            out.append(cb)
        if return_disentangled:
            out.append(self.cond_stage_model.encoding(xc) if hasattr(self.cond_stage_model, "encoding") else None)
        return out

    def shared_step(self, batch, **kwargs):
        x, c = self.get_input(batch, self.first_stage_key)
        return self(x, c)

    def forward(self, x, c, *args, **kwargs):
        """ddpm_enc.py:1040-1053."""
        t = torch.randint(0, self.num_timesteps, (x.shape[0],), device=self.device).long()
        if self.model.conditioning_key is not None and self.cond_stage_trainable:
            c = self.get_learned_conditioning(c)
        return self.p_losses(x, c, t, *args, **kwargs)

    def apply_model(self, x_noisy, t, cond, return_ids=False, return_context=False):
        """ddpm_enc.py:1065-1163 (no split_input_params path)."""
        if isinstance(cond, dict):
            pass
        else:
            if not isinstance(cond, list):
                cond = [cond]
            key = "c_concat" if self.model.conditioning_key == "concat" else "c_crossattn"
            cond = {key: cond}
        return self.model(x_noisy, t, **cond)

    def p_losses(self, x_start, cond, t, noise=None):
        """ddpm_enc.py:1183-1253 (eps parameterisation, L1, logvar == 0)."""
        if self.parameterization != "eps" or self.loss_type != "l1" or self.learn_logvar:
            raise NotImplementedError("HIP p_losses covers the EncDiff objective (eps, l1, fixed logvar)")
        noise = default(noise, lambda: torch.randn_like(x_start))
        x_noisy = self.q_sample(x_start, t, noise)
        model_output = self.apply_model(x_noisy, t, cond)
        prefix = "train" if self.training else "val"
        loss, loss_vlb = _PLossFn.apply(model_output, noise, t, self.lvlb_weights, float(self.l_simple_weight))
        loss_simple = loss / float(self.l_simple_weight) if self.l_simple_weight else loss
        # logvar == logvar_init == 0: loss = loss_simple/exp(0) + 0 (ddpm_enc.py:1202-1208)
        loss = loss + self.original_elbo_weight * loss_vlb
        loss_dict = {f"{prefix}/loss_simple": loss_simple.detach(), f"{prefix}/loss_vlb": loss_vlb.detach(),
                     f"{prefix}/loss": loss.detach(), f"{prefix}/epoch_num": self.current_epoch}
        return loss, loss_dict

    # ------------------------------------------------------------ HIP training setup
    def hip_trainables(self):
        """Arena order: UNet params (EMA-tracked, fused-group layout) then the cond stage."""
        unet = self.model.diffusion_model
        order = [("model.diffusion_model." + n, p) for n, p in unet.arena_order()]
        if self.cond_stage_trainable and self.cond_stage_model is not None:
            order += [("cond_stage_model." + n, p) for n, p in self.cond_stage_model.named_parameters()]
        return order

    def setup_hip_training(self):
        """Build the shared parameter arena, bind the UNet executor and the EMA to it."""
        from encdiff_amd.arena import ParamArena
        unet = self.model.diffusion_model
        order = self.hip_trainables()
        ema_names = ["model.diffusion_model." + n for n, _ in unet.named_parameters()]
        cl = ["model.diffusion_model." + n for n in unet._spec.conv_weights()]
        cs = self.cond_stage_model
        if self.cond_stage_trainable and type(cs).__name__ == "Encoder4":
            from encdiff_amd.cond import Encoder4TrunkExecutor   # trunk convs channels-last (§8(f) row 2)
            cl += Encoder4TrunkExecutor.channels_last_names(cs, "cond_stage_model.")
        arena = ParamArena(order, self.device, ema_names=ema_names, channels_last=cl)

        # the UNet executor addresses its parameters by their UNet-local names
        for n in list(arena.offsets):
            if n.startswith("model.diffusion_model."):
                arena.alias(n[len("model.diffusion_model."):], n)
        unet.bind_arena(arena)
        fs = self.first_stage_model
        if hasattr(fs, "enable_hip") and getattr(fs, "_hip_encoder", None) is None:
            fs.enable_hip()                              # frozen VQ encoder on HIP (§8(f) row 2)
        cs = self.cond_stage_model
        if self.cond_stage_trainable and cs is not None and hasattr(cs, "bind_arena"):
            cs.bind_arena(arena, "cond_stage_model.")   # Encoder4.warp on HIP (§8(f) row 2)
        if self.use_ema:
            self.model_ema.bind_arena(arena, prefix="model.")
            self._ema_fused = True
        self._arena = arena
        return arena

    def configure_optimizers(self):
        """ddpm_enc.py:1598-1639: AdamW over UNet (+ cond stage) params, LambdaLR per step."""
        lr = getattr(self, "learning_rate", 1e-4)
        if getattr(self, "_arena", None) is None:
            self.setup_hip_training()
        arena = self._arena
        unet = self.model.diffusion_model
        params = [p for _, p in self.hip_trainables()]
        rp_unet = lambda: (unet.executor().pack.repack(), unet.mark_repacked())  # noqa: E731
        rp_cond = lambda: getattr(self.cond_stage_model, "repack_hip", lambda: None)()  # noqa: E731
        opt = FusedArenaAdamW(params, arena, lr=lr, ema=self.model_ema if self.use_ema else None,
                              repack=lambda: (rp_unet(), rp_cond()), repack_parts=(rp_unet, rp_cond))
        self._optimizer = opt
        if self.use_scheduler:
            sched = instantiate_from_config(self.scheduler_config)
            return [opt], [{"scheduler": torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=sched.schedule),
                            "interval": "step", "frequency": 1}]
        return opt

    # ------------------------------------------------------------ sampling
    def ddim_sampler(self):
        """One DDIMSampler per model: its captured loop graphs (keyed by batch shape, S, eta,
        log_every_t) are reused by every later log_images / sample_log / sample_swap call."""
        s = getattr(self, "_ddim_sampler", None)
        if s is None:
            s = self._ddim_sampler = DDIMSampler(self)
        return s

    @torch.no_grad()
    def sample_log(self, cond, batch_size, ddim, ddim_steps, **kwargs):
        if not ddim:
            raise NotImplementedError("ancestral p_sample loop is not on the EncDiff path; use ddim=True")
        sampler = self.ddim_sampler()
        shape = (self.channels, self.image_size, self.image_size)
        return sampler.sample(ddim_steps, batch_size, shape, cond, verbose=False, **kwargs)

    @torch.no_grad()
    def sample_swap(self, orc, N, ddim_steps=200, eta=1., x_T=None, normals_sequence=None):
        """The log_images sample_swap workload (ddpm_enc.py:1522-1535) as ONE sampler run: for
        every concept unit cdx the batch's scalar codes `orc` (B, latent_unit) get unit cdx
        replaced by the first image's, are warped to concept tokens, and sampled with DDIM.
        The reference runs latent_unit separate DDIM loops of batch N; the UNet treats every
        sample independently (per-sample GroupNorm, attention within a sample), so the
        latent_unit x N conditionings are stacked into one (latent_unit * N) batch and sampled by
        one captured loop.  Returns latents (latent_unit * N, C, H, W), row-block cdx = the
        reference's cdx-th call."""
        lu = self.model.diffusion_model.latent_unit
        orc = orc[:N]
        n = orc.shape[0]
        sc = orc[None].repeat(lu, 1, 1)                       # [cdx][b][unit]
        idx = torch.arange(lu, device=orc.device)
        sc[idx, :, idx] = orc[0][:, None].expand(lu, n)       # unit cdx <- image 0's unit cdx
        cond = self.cond_stage_model.warp(sc.reshape(lu * n, lu))
        shape = (self.channels, self.image_size, self.image_size)
        sampler = self.ddim_sampler()
        samples, _ = sampler.sample(ddim_steps, lu * n, shape, cond.reshape(lu * n, -1), eta=eta, verbose=False,
                                    x_T=x_T, normals_sequence=normals_sequence)
        return samples

    # ------------------------------------------------------------ validation (§8(f) row 4)
    @torch.no_grad()
    def validation_step(self, batch, batch_idx=0):
        """ddpm_enc.py:377-390: concept tokens c (B, latent_unit, context_dim) and scalar codes
        orc (B, latent_unit) of the batch, collected for the epoch-end metrics (eval_func is
        out of scope; on_validation_epoch_end returns the stacked arrays)."""
        x, oc = self.get_input(batch, self.first_stage_key)
        c, orc = self.encode_concepts(oc)
        if not hasattr(self, "validation_step_outputs"):
            self.validation_step_outputs, self.validation_step_scalars = [], []
        self.validation_step_outputs.append(c.detach().cpu().numpy())
        self.validation_step_scalars.append(orc.detach().cpu().numpy())

    def on_validation_epoch_end(self, *args, **kwargs):
        """Returns (codes (N, latent_unit), tokens (N, latent_unit, context_dim)) -- what the
        reference hands to eval_func (ddpm_enc.py:403-425) -- and clears the lists."""
        outs = getattr(self, "validation_step_outputs", [])
        scal = getattr(self, "validation_step_scalars", [])
        res = (np.concatenate(scal, 0) if scal else None, np.concatenate(outs, 0) if outs else None)
        if outs:
            outs.clear()
            scal.clear()
        return res

    @torch.no_grad()
    def encode_concepts(self, img):
        """Encoder4 in eval mode (running BatchNorm statistics): tokens c (B, latent_unit,
        context_dim) = warp(orc) and codes orc (B, latent_unit)."""
        cs = self.cond_stage_model
        was = cs.training
        cs.eval()
        try:
            orc = cs.encoding(img)
            c = cs.warp(orc)
        finally:
            cs.train(was)
        return c.reshape(c.shape[0], self.model.diffusion_model.latent_unit, -1), orc

    @torch.no_grad()
    def encode_dataset(self, pool, chunk=4096):
        """Validation encoding pass over a GPU-resident uint8 image pool
        (encdiff_amd.data.ImagePool, or a uint8 [N, H, W, C] device tensor): fused
        gather + ToTensor/Normalize, the HIP Encoder4 trunk in eval mode, Linear and the warp
        MLPs, `chunk` images per pass, results kept on the device.  Returns (codes (N,
        latent_unit), tokens (N, latent_unit, context_dim)) in dataset order -- the arrays the
        reference collects batch by batch through validation_step (ddpm_enc.py:377-390)."""
        images = pool.images if hasattr(pool, "images") else pool
        n = images.shape[0]
        dev = images.device
        lu = self.model.diffusion_model.latent_unit
        cd = self.cond_stage_model.context_dim
        codes = torch.empty(n, lu, device=dev)
        toks = torch.empty(n, lu, cd, device=dev)
        order = torch.arange(n, device=dev, dtype=torch.int64)
        for s in range(0, n, chunk):
            b = min(chunk, n - s)
            img = torch.empty(b, images.shape[3], images.shape[1], images.shape[2], device=dev)
            step = torch.zeros(1, device=dev, dtype=torch.int64)
            ops.gather_images_u8(images, order[s:s + b], step, b, img, advance=False)
            c, orc = self.encode_concepts(img)
            codes[s:s + b].copy_(orc)
            toks[s:s + b].copy_(c)
        return codes, toks

    @torch.no_grad()
    def log_images(self, batch, N=8, n_row=4, sample=True, ddim_steps=200, ddim_eta=1., return_keys=None,
                   quantize_denoised=True, inpaint=True, plot_denoise_rows=False, plot_progressive_rows=True,
                   sample_swap=False, plot_diffusion_rows=True, **kwargs):
        """ddpm_enc.py:1473-1596: inputs, reconstruction, diffusion row, swap samples and samples
        (DDIM); inpainting / progressive rows are not on the EncDiff path."""
        log = {}
        z, c, x, xrec, xc, orc = self.get_input(batch, self.first_stage_key, return_first_stage_outputs=True,
                                                force_c_encode=True, return_original_cond=True, bs=N,
                                                return_false=True)
        N = min(x.shape[0], N)
        n_row = min(x.shape[0], n_row)
        log["inputs"], log["reconstruction"] = x, xrec
        if plot_diffusion_rows:
            rows = []
            z_start = z[:n_row]
            for t in range(self.num_timesteps):
                if t % self.log_every_t == 0 or t == self.num_timesteps - 1:
                    tt = torch.full((n_row,), t, device=self.device, dtype=torch.long)
                    rows.append(self.decode_first_stage(self.q_sample(z_start, tt, torch.randn_like(z_start))))
            log["diffusion_row"] = torch.stack(rows)
        if sample_swap:
            with self.ema_scope("Plotting Swapping"):
                log["samples_swapping"] = self.decode_first_stage(
                    self.sample_swap(orc, N, ddim_steps=ddim_steps, eta=ddim_eta))
        if sample:
            with self.ema_scope("Plotting"):
                samples, _ = self.sample_log(cond=c, batch_size=N, ddim=True, ddim_steps=ddim_steps, eta=ddim_eta)
            log["samples"] = self.decode_first_stage(samples)
        if return_keys:
            return {k: v for k, v in log.items() if k in return_keys}
        return log


class DiffusionWrapper(nn.Module):
    """ddpm_enc.py:1651-1677."""

    def __init__(self, diff_model_config, conditioning_key):
        super().__init__()
        self.diffusion_model = instantiate_from_config(diff_model_config)
        self.conditioning_key = conditioning_key
        assert conditioning_key in [None, "concat", "crossattn", "hybrid", "adm"]

    def forward(self, x, t, c_concat: list = None, c_crossattn: list = None, return_context=False):
        if self.conditioning_key is None:
            return self.diffusion_model(x, t, context=c_crossattn[0])
        if self.conditioning_key == "crossattn":
            return self.diffusion_model(x, t, context=c_crossattn)
        raise NotImplementedError(f"conditioning_key {self.conditioning_key} is not on the EncDiff path")
