"""Checker of the benchmarked training step (TEST INFRASTRUCTURE -- imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product path).

Runs the graph-captured ``encdiff_amd.trainer.HipTrainer`` -- the object bench.py times --
with recipe weights (every layer non-zero, so eps and all gradients carry data) and feeds each
replay's image batch, timesteps and noise through ``HipTrainer.enable_feed()``.  The CPU oracle
(``OracleTrainer``: fp32, VQ encode, training-mode Encoder4, q_sample, UNet, L1, AdamW, EMA)
starts from the trainer's state after its eager warm-up steps and runs the same inputs.

Reference: ddpm_enc.py:360-375 (training_step), :773-844 (get_input), :1040-1053 (forward),
:1183-1253 (p_losses), :1598-1639 (AdamW), ema.py:25-44 (LitEma).

Tolerances (bf16 activations vs the fp32 reference): eps rel-L2 <= 3e-2 and
max-abs <= 6e-2; loss rel <= 1e-2; gradients rel-L2 <= 5e-2; AdamW / EMA parameter updates
rel-L2 <= 5e-2.  The L1 gradient seed sign(eps - noise)/N is discontinuous, so the oracle
back-propagates the seed the device computed (derived from the device eps); the loss value is
compared separately.
"""
from __future__ import annotations

import torch

from . import encdiff_oracle as O

TOL = dict(eps_rel=3e-2, eps_max=6e-2, loss_rel=1e-2, grad_rel=5e-2, update_rel=5e-2)

# UNet: every block type, the producer-statistics GroupNorms and the LN epilogues
GRAD_NAMES = [
    "time_embed.0.weight", "time_embed.2.weight", "input_blocks.0.0.weight",
    "input_blocks.1.0.in_layers.2.weight", "input_blocks.1.0.emb_layers.1.weight",
    "input_blocks.1.1.proj_in.weight", "input_blocks.1.1.transformer_blocks.0.attn1.to_q.weight",
    "input_blocks.1.1.transformer_blocks.0.attn2.to_k.weight",
    "input_blocks.1.1.transformer_blocks.0.ff.net.0.proj.weight",
    "input_blocks.1.1.transformer_blocks.0.norm1.weight", "input_blocks.3.0.in_layers.2.weight",
    "input_blocks.4.0.skip_connection.weight", "input_blocks.7.1.norm.weight",
    "middle_block.1.transformer_blocks.0.attn1.to_out.0.weight", "middle_block.2.out_layers.3.weight",
    "output_blocks.2.1.in_layers.2.weight", "output_blocks.5.1.transformer_blocks.0.norm3.bias",
    "output_blocks.8.2.out_layers.0.weight", "output_blocks.11.1.proj_out.weight",
    "output_blocks.11.0.skip_connection.weight", "out.0.weight", "out.2.weight",
]
COND_NAMES = ["encoder.0.weight", "encoder.3.weight", "encoder.9.weight", "encoder.11.convs.1.weight",
              "encoder.14.convs.4.weight", "encoder.16.weight", "net.3.2.weight", "net.17.4.weight"]


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def recipe_ldm(config="shapes3d", unet_params=None):
    """LatentDiffusion from the reference-shaped config with recipe weights in the UNet,
    Encoder4 and the VQ first stage, on cuda.  ``unet_params`` overrides UNetModel kwargs
    (e.g. ``attn_fp8_min_tokens``) for this instance only."""
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    cfg = model_config(config)
    if unet_params:
        cfg["params"]["unet_config"]["params"].update(unet_params)
    torch.manual_seed(0)
    ldm = instantiate_from_config(cfg)
    with torch.no_grad():
        for n, p in ldm.model.diffusion_model.named_parameters():
            p.copy_(O.recipe_tensor(n, tuple(p.shape)))
        for n, p in ldm.cond_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("cond." + n, tuple(p.shape)))
        for n, p in ldm.first_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("vq." + n, tuple(p.shape)))
    return ldm.cuda(), cfg


class GraphStepCheck:
    """HipTrainer (graph replay, fed inputs) vs OracleTrainer on identical inputs.

    ``config``: "shapes3d" (configs[1] / configs[3] shapes) or "celeba128" (configs[4]).
    ``check()`` runs one replay + one oracle step and returns the error dict; the oracle
    then adopts the device parameters so that the next check starts from identical state."""

    def __init__(self, B=128, config="shapes3d", lr=1e-4, seed=2024, warmup=2, threads=16, unet_params=None,
                 oracle_scale=True):
        from encdiff_amd.trainer import HipTrainer
        torch.set_num_threads(max(1, min(threads, torch.get_num_threads())))
        self.B, self.config = B, config
        ldm, cfg = recipe_ldm(config, unet_params)
        ucfg = cfg["params"]["unet_config"]["params"]
        self.lu = ucfg["latent_unit"]
        self.res = 64 if config == "shapes3d" else 128
        self.zres = self.res // 4
        self.ldm = ldm
        # constant lr (the recipe's LambdaLinearScheduler starts at 1e-6 x lr, which would make
        # the AdamW update numerically empty); lr = B * base_lr as main_val.py:834-838
        ldm.use_scheduler = False
        self.tr = tr = HipTrainer(ldm, B, base_lr=lr / B, graph=True, pool_size=2 * B)
        self.feed = tr.enable_feed()
        self.g = torch.Generator().manual_seed(seed)
        img, t, noise = self.inputs()
        self._put(img, t, noise)
        tr.init_scale_factor()
        self.sf_hip = float(ldm.scale_factor)
        tr.capture(warmup=warmup)  # eager steps, then the graph the benchmark replays
        torch.cuda.synchronize()
        a = tr.arena
        plan = O.build_plan(ucfg)
        self.unet_names = list(O.param_shapes(plan))
        self.cond_names = [n for n in O.encoder4_shapes(latent_unit=self.lu, image_size=self.res)
                           if "running" not in n and "num_batches" not in n]
        v = self._view
        m = {n: v(a.exp_avg, n) for n in self.unet_names}
        s = {n: v(a.exp_avg_sq, n) for n in self.unet_names}
        m.update({"cond." + n: v(a.exp_avg, "cond_stage_model." + n) for n in self.cond_names})
        s.update({"cond." + n: v(a.exp_avg_sq, "cond_stage_model." + n) for n in self.cond_names})
        self.orc = orc = O.OracleTrainer(plan, lr=lr, vq=True, image_size=self.res)
        orc.load_state({n: v(a.master, n) for n in self.unet_names},
                       {n: v(a.master, "cond_stage_model." + n) for n in self.cond_names}, m, s,
                       tr.opt.step_count, {n: v(a.ema, n) for n in self.unet_names},
                       int(ldm.model_ema.num_updates))
        # scale_by_std (ddpm_enc.py:586-608) on the oracle's own fp32 latents of the first batch
        # (oracle_scale=False: adopt the device's -- a whole-batch statistic, and the VQ encode of a
        # large batch of 128x128 images is what a CPU oracle cannot afford; check_rows)
        with torch.no_grad():
            orc.scale_factor = (float(1.0 / O.vq_encode(orc.V, img).flatten().std()) if oracle_scale
                                else self.sf_hip)

    def _view(self, buf, n):
        return self.tr.arena.view_in(buf, n).detach().cpu().clone()

    def inputs(self):
        B, g = self.B, self.g
        u8 = torch.randint(0, 256, (B, self.res, self.res, 3), generator=g, dtype=torch.uint8)
        return (O.images_to_input(u8, torch.arange(B)), torch.randint(0, 1000, (B,), generator=g),
                torch.randn(B, 3, self.zres, self.zres, generator=g))

    def _put(self, img, t, noise):
        self.feed["img"].copy_(img)
        self.feed["t"].copy_(t)
        self.feed["noise"].copy_(noise)

    def check(self, grad_names=GRAD_NAMES, cond_names=COND_NAMES):
        tr, orc, a = self.tr, self.orc, self.tr.arena
        names, cnames = self.unet_names, self.cond_names
        img, t, noise = self.inputs()
        self._put(img, t, noise)
        before = {n: self._view(a.master, n) for n in names}
        ema_before = {n: self._view(a.ema, n) for n in names}
        cond_before = {n: self._view(a.master, "cond_stage_model." + n) for n in cnames}
        tr.step()  # graph replay: the benchmarked step
        torch.cuda.synchronize()
        eps = tr.eps().detach().cpu().clone()
        loss = tr.loss()
        seed = torch.sign(eps - noise) / eps.numel()
        o_before = {n: p.detach().clone() for n, p in orc.P.items()}
        lo = float(orc.step_images(img, t, noise, seed=seed))
        oeps = orc.last["eps"]
        r = dict(B=self.B, config=self.config, eps_rel=rel(eps, oeps), eps_max=(eps - oeps).abs().max().item(),
                 loss=loss, loss_oracle=lo, loss_rel=abs(loss - lo) / lo)
        # the device loss is the L1 of the device eps, exact up to summation order
        host = (eps.double() - noise.double()).abs().mean().item()
        r["loss_vs_device_eps"] = abs(loss - host) / host
        gl = {n: rel(a.view_in(a.grad, n), orc.P[n].grad) for n in grad_names if n in orc.P}
        gl.update({"cond." + n: rel(a.view_in(a.grad, "cond_stage_model." + n), orc.E[n].grad)
                   for n in cond_names if n in orc.E})
        r["grads_listed"] = gl
        worst = max(((rel(a.view_in(a.grad, n), orc.P[n].grad), n) for n in names if orc.P[n].grad.norm() > 0))
        r["worst_unet_grad"] = worst
        gh = torch.cat([a.view_in(a.grad, n).detach().cpu().flatten() for n in names])
        go = torch.cat([orc.P[n].grad.flatten() for n in names])
        r["unet_grads_rel"] = rel(gh, go)
        ch = torch.cat([a.view_in(a.grad, "cond_stage_model." + n).detach().cpu().flatten() for n in cnames])
        co = torch.cat([orc.E[n].grad.flatten() for n in cnames])
        r["cond_grads_rel"] = rel(ch, co)
        # AdamW update and EMA update (fp64 differences of fp32 values)
        dh = torch.cat([(self._view(a.master, n).double() - before[n].double()).flatten() for n in names])
        do = torch.cat([(orc.P[n].detach().double() - o_before[n].double()).flatten() for n in names])
        eh = torch.cat([(self._view(a.ema, n).double() - ema_before[n].double()).flatten() for n in names])
        eo = torch.cat([(orc.ema[n].double() - ema_before[n].double()).flatten() for n in names])
        cu = torch.cat([(self._view(a.master, "cond_stage_model." + n).double() - cond_before[n].double()).flatten()
                        for n in cnames])
        cuo = torch.cat([(orc.E[n].detach().double() - cond_before[n].double()).flatten() for n in cnames])
        r.update(adamw_rel=rel(dh, do), ema_rel=rel(eh, eo), cond_adamw_rel=rel(cu, cuo))
        # the two runs now differ by these updates only: carry the device state into the oracle
        with torch.no_grad():
            for n, p in orc.P.items():
                p.copy_(a.view_in(a.master, n).detach().cpu())
            for n in cnames:
                orc.E[n].copy_(a.view_in(a.master, "cond_stage_model." + n).detach().cpu())
            for n in names:
                orc.ema[n].copy_(a.view_in(a.ema, n).detach().cpu())
        return r


    def check_rows(self, rows):
        """The benchmarked step at a batch a full CPU oracle step cannot finish in test time: one
        graph replay, then the oracle FORWARD of the listed rows only -- the VQ encode, q_sample and
        the UNet are per image; Encoder4's training-mode BatchNorm couples the batch, so it runs on
        all B images and the rows' concept tokens are taken from it -- vs the device eps of those
        rows (eps tolerances).  Batch-level properties beside it: the device loss is the L1 of the
        device eps of all B images, and every UNet / Encoder4 gradient and parameter update is
        finite and non-zero."""
        tr, orc, a = self.tr, self.orc, self.tr.arena
        img, t, noise = self.inputs()
        self._put(img, t, noise)
        before = a.master.detach().clone()
        tr.step()
        torch.cuda.synchronize()
        eps = tr.eps().detach().cpu().clone()
        loss = tr.loss()
        idx = torch.as_tensor(rows, dtype=torch.long)
        with torch.no_grad():
            c = O.encoder4_forward(orc.E, img, latent_unit=orc.lu)
            x0 = orc.scale_factor * O.vq_encode(orc.V, img[idx])
            xn = O.q_sample(orc.sched, x0, t[idx], noise[idx])
            oeps = O.unet_forward(orc.P, orc.plan, xn, t[idx], [c[idx]])
        host = (eps.double() - noise.double()).abs().mean().item()
        g = a.grad.detach()
        upd = (a.master.detach() - before)
        unet_n = a.ema_numel
        return dict(B=self.B, config=self.config, rows=list(rows), eps_rel=rel(eps[idx], oeps),
                    eps_max=(eps[idx] - oeps).abs().max().item(), loss=loss,
                    loss_vs_device_eps=abs(loss - host) / host,
                    grads_finite=bool(torch.isfinite(g).all()),
                    unet_grad_norm=float(g[:unet_n].norm()), cond_grad_norm=float(g[unet_n:].norm()),
                    update_finite=bool(torch.isfinite(upd).all()), update_norm=float(upd.norm()))


def failures(r, tol=TOL, every_param=False):
    """Names of the tolerance checks ``r`` (from GraphStepCheck.check) fails.  ``every_param``
    also holds the worst single UNet parameter gradient to the gradient tolerance."""
    bad = []
    if not (r["eps_rel"] < tol["eps_rel"] and r["eps_max"] < tol["eps_max"]):
        bad.append("eps")
    if not r["loss_vs_device_eps"] < 1e-5:
        bad.append("loss_vs_device_eps")
    if not r["loss_rel"] < tol["loss_rel"]:
        bad.append("loss")
    for k, v in r["grads_listed"].items():
        if not v < tol["grad_rel"]:
            bad.append("grad:" + k)
    if every_param and not r["worst_unet_grad"][0] < tol["grad_rel"]:
        bad.append("worst_unet_grad:" + r["worst_unet_grad"][1])
    for k in ("unet_grads_rel", "cond_grads_rel"):
        if not r[k] < tol["grad_rel"]:
            bad.append(k)
    for k in ("adamw_rel", "ema_rel", "cond_adamw_rel"):
        if not r[k] < tol["update_rel"]:
            bad.append(k)
    return bad


def summary(r):
    return (f"{r['config']} B={r['B']}: eps rel-L2 {r['eps_rel']:.3e} max-abs {r['eps_max']:.3e}; "
            f"loss {r['loss']:.5f} vs {r['loss_oracle']:.5f}; UNet grads {r['unet_grads_rel']:.3e} "
            f"(worst {r['worst_unet_grad'][1]} {r['worst_unet_grad'][0]:.3e}); Encoder4 grads "
            f"{r['cond_grads_rel']:.3e}; AdamW {r['adamw_rel']:.3e} / Encoder4 {r['cond_adamw_rel']:.3e}; "
            f"EMA {r['ema_rel']:.3e}")
