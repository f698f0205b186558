"""DDIMSampler -- mirror of ldm/models/diffusion/ddim.py:11-207 on the HIP path.

Same schedule construction (make_schedule, :24-54), same sampling loop order and
noise consumption (one N(0, I) draw of x's shape per step, :201), same update
(p_sample_ddim, :188-207) -- the update itself is one HIP kernel.

With ``use_graph=True`` (default on a HIP device, when no per-step callbacks, masks or
guidance are requested) the WHOLE S-step loop -- S x (UNet forward + DDIM update), plus
the copies of the logged intermediates -- is captured into one HIP graph per (batch shape,
S, eta, log_every_t) and replayed once per ``sample()`` call.  Everything the graph reads
lives in buffers owned by its cache entry (x_T, the conditioning, the per-step noise table,
the timestep rows), so a later call with other inputs copies them in and replays; the
schedule coefficients are kernel arguments of the unrolled steps.  Loops longer than
``GRAPH_MAX_STEPS`` capture one step (coefficients and timestep looked up at a device step
index) and replay it S times.

Noise: with eta > 0 each captured step draws its N(0, I) row inside the graph (torch's
graph-safe Philox stream advances on every replay), so a loop holds one step's noise, not an
(S, *x.shape) table.  ``normals_sequence`` (the reference's kwarg, unused there) injects a
given table instead -- step i (in loop order, i = 0 .. S-1) adds sigma_i * normals_sequence[i]
-- which is how the eta > 0 trajectory is pinned against the reference's CPU noise stream.
At eta == 0 sigma is 0 for every step and no noise is drawn.

Before a replay the model's bf16 weight packs are refreshed if the parameters changed in
place since the capture (LatentDiffusion.refresh_hip_weights): a sampler captured outside
ema_scope() samples with the EMA weights inside it.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from encdiff_amd import ops, torch_ops  # noqa: F401  (torch_ops registers torch.ops.encdiff.*)
from ...modules.diffusionmodules.util import make_ddim_sampling_parameters, make_ddim_timesteps, noise_like

GRAPH_MAX_STEPS = 256  # longer loops replay a one-step graph (device step index)
# Capturing a whole S-step loop records S x ~300 kernel nodes (~4 s at S = 200), which only pays
# when the same (batch shape, S, eta) is sampled again: the first LOOP_GRAPH_AFTER calls of a
# loop replay the one-step graph (captured in milliseconds, ~1 % slower per step), later calls
# capture and replay the whole-loop graph.  A one-off call (the first log_images) then costs
# about its sampling time; repeated sampling (validation, the bench) runs the loop graph.
LOOP_GRAPH_AFTER = 1
# whole-loop graph: K / V of the conditioning and the FiLM rows of all steps computed once per loop
HOIST = os.environ.get("ENCDIFF_DDIM_HOIST", "1") != "0"


class DDIMSampler(object):
    def __init__(self, model, schedule="linear", use_graph=True, **kwargs):
        super().__init__()
        self.model = model
        self.ddpm_num_timesteps = model.num_timesteps
        self.schedule = schedule
        self.use_graph = use_graph
        self._graphs = {}
        self._seen = {}  # loop key -> sample() calls so far (LOOP_GRAPH_AFTER)
        # (S, eta) -> device coefficient / timestep tables.  Allocated once and kept: a
        # captured graph holds their addresses, so they are never rebound or freed.
        self._tables = {}

    def register_buffer(self, name, attr):
        if isinstance(attr, torch.Tensor):
            attr = attr.to(self.model.device)
        setattr(self, name, attr)

    def make_schedule(self, ddim_num_steps, ddim_discretize="uniform", ddim_eta=0., verbose=True):
        self.ddim_timesteps = make_ddim_timesteps(ddim_discretize, ddim_num_steps, self.ddpm_num_timesteps,
                                                  verbose=verbose)
        alphas_cumprod = self.model.alphas_cumprod
        assert alphas_cumprod.shape[0] == self.ddpm_num_timesteps
        to_t = lambda x: x.clone().detach().to(torch.float32).to(self.model.device)  # noqa: E731
        self.register_buffer("betas", to_t(self.model.betas))
        self.register_buffer("alphas_cumprod", to_t(alphas_cumprod))
        self.register_buffer("alphas_cumprod_prev", to_t(self.model.alphas_cumprod_prev))
        ac = alphas_cumprod.cpu()
        self.register_buffer("sqrt_alphas_cumprod", to_t(torch.sqrt(ac)))
        self.register_buffer("sqrt_one_minus_alphas_cumprod", to_t(torch.sqrt(1. - ac)))
        sig, a, ap, an = make_ddim_sampling_parameters(ac, self.ddim_timesteps, ddim_eta, verbose=verbose)
        self.ddim_sigmas, self.ddim_alphas, self.ddim_alphas_prev, self.ddim_alphas_next = sig, a, ap, an
        self.ddim_sqrt_one_minus_alphas = np.sqrt(1. - a)
        self.ddim_eta = ddim_eta
        key = (ddim_discretize, int(ddim_num_steps), float(ddim_eta))
        tab = self._tables.get(key)
        if tab is None:
            # coef[index] = (a_t, a_prev, sigma, sqrt(1 - a_t)); ts[index]
            coef = np.stack([a, ap, sig, self.ddim_sqrt_one_minus_alphas], axis=1).astype(np.float32)
            tab = self._tables[key] = (torch.tensor(coef, device=self.model.device),
                                       torch.tensor(np.asarray(self.ddim_timesteps, dtype=np.int64),
                                                    device=self.model.device))
        self._coef, self._ts = tab
        self._sched_key = key

    @torch.no_grad()
    def sample(self, S, batch_size, shape, conditioning=None, callback=None, normals_sequence=None,
               img_callback=None, quantize_x0=False, eta=0., mask=None, x0=None, temperature=1.,
               noise_dropout=0., score_corrector=None, corrector_kwargs=None, verbose=True, x_T=None,
               log_every_t=100, unconditional_guidance_scale=1., unconditional_conditioning=None, **kwargs):
        self.make_schedule(ddim_num_steps=S, ddim_eta=eta, verbose=verbose)
        C, H, W = shape
        size = (batch_size, C, H, W)
        return self.ddim_sampling(conditioning, size, callback=callback, img_callback=img_callback,
                                  quantize_denoised=quantize_x0, mask=mask, x0=x0, temperature=temperature,
                                  noise_dropout=noise_dropout, score_corrector=score_corrector,
                                  corrector_kwargs=corrector_kwargs, x_T=x_T, log_every_t=log_every_t,
                                  unconditional_guidance_scale=unconditional_guidance_scale,
                                  unconditional_conditioning=unconditional_conditioning,
                                  normals_sequence=normals_sequence)

    @torch.no_grad()
    def ddim_sampling(self, cond, shape, x_T=None, ddim_use_original_steps=False, callback=None, timesteps=None,
                      quantize_denoised=False, mask=None, x0=None, img_callback=None, log_every_t=100,
                      temperature=1., noise_dropout=0., score_corrector=None, corrector_kwargs=None,
                      unconditional_guidance_scale=1., unconditional_conditioning=None, normals_sequence=None):
        device = self.model.betas.device
        b = shape[0]
        img = torch.randn(shape, device=device) if x_T is None else x_T.to(device).float().contiguous()
        if ddim_use_original_steps:
            raise NotImplementedError("ddim_use_original_steps is not used by EncDiff")
        if timesteps is not None:
            end = int(min(timesteps / self.ddim_timesteps.shape[0], 1) * self.ddim_timesteps.shape[0]) - 1
            steps = self.ddim_timesteps[:end]
        else:
            steps = self.ddim_timesteps
        total = steps.shape[0]
        if normals_sequence is not None:
            normals_sequence = self._noise_table(normals_sequence, total, img.shape, device)
        intermediates = {"x_inter": [img], "pred_x0": [img]}
        simple = (callback is None and img_callback is None and mask is None and not quantize_denoised and
                  noise_dropout == 0. and score_corrector is None and temperature == 1. and
                  (unconditional_conditioning is None or unconditional_guidance_scale == 1.))
        if self.use_graph and simple and img.is_cuda and timesteps is None and isinstance(cond, torch.Tensor):
            if total <= GRAPH_MAX_STEPS:
                lk = (tuple(img.shape), total, self._sched_key, tuple(cond.shape), cond.dtype, log_every_t,
                      bool(normals_sequence is not None and self.ddim_eta))
                seen = self._seen.get(lk, 0)
                self._seen[lk] = seen + 1
                if seen >= LOOP_GRAPH_AFTER:
                    return self._loop_graph(cond, img, total, log_every_t, intermediates, normals_sequence)
            return self._step_graph(cond, img, total, log_every_t, intermediates, normals_sequence)
        for i, step in enumerate(np.flip(steps)):
            index = total - i - 1
            ts = torch.full((b,), int(step), device=device, dtype=torch.long)
            if mask is not None:
                img = self.model.q_sample(x0, ts) * mask + (1. - mask) * img
            img, pred_x0 = self.p_sample_ddim(img, cond, ts, index=index, quantize_denoised=quantize_denoised,
                                              temperature=temperature, noise_dropout=noise_dropout,
                                              score_corrector=score_corrector, corrector_kwargs=corrector_kwargs,
                                              unconditional_guidance_scale=unconditional_guidance_scale,
                                              unconditional_conditioning=unconditional_conditioning,
                                              noise=None if normals_sequence is None else normals_sequence[i])
            if callback:
                callback(i)
            if img_callback:
                img_callback(pred_x0, i)
            if index % log_every_t == 0 or index == total - 1:
                intermediates["x_inter"].append(img)
                intermediates["pred_x0"].append(pred_x0)
        return img, intermediates

    @staticmethod
    def _noise_table(seq, total, shape, device):
        t = torch.stack(list(seq)) if not isinstance(seq, torch.Tensor) else seq
        t = t.to(device=device, dtype=torch.float32).contiguous()
        if t.shape[0] < total or tuple(t.shape[1:]) != tuple(shape):
            raise ValueError(f"normals_sequence must hold {total} draws of shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    @torch.no_grad()
    def p_sample_ddim(self, x, c, t, index, repeat_noise=False, use_original_steps=False, quantize_denoised=False,
                      temperature=1., noise_dropout=0., score_corrector=None, corrector_kwargs=None,
                      unconditional_guidance_scale=1., unconditional_conditioning=None, noise=None):
        b = x.shape[0]
        if unconditional_conditioning is None or unconditional_guidance_scale == 1.:
            e_t = self.model.apply_model(x, t, c)
        else:
            x_in, t_in = torch.cat([x] * 2), torch.cat([t] * 2)
            c_in = torch.cat([unconditional_conditioning, c])
            e_u, e_t = self.model.apply_model(x_in, t_in, c_in).chunk(2)
            e_t = e_u + unconditional_guidance_scale * (e_t - e_u)
        if score_corrector is not None:
            e_t = score_corrector.modify_score(self.model, e_t, x, t, c, **corrector_kwargs)
        a_t, a_prev = float(self.ddim_alphas[index]), float(self.ddim_alphas_prev[index])
        sigma, s1 = float(self.ddim_sigmas[index]), float(self.ddim_sqrt_one_minus_alphas[index])
        if noise is None:
            noise = noise_like(x.shape, x.device, repeat_noise)
        noise = noise * temperature
        if noise_dropout > 0.:
            noise = torch.nn.functional.dropout(noise, p=noise_dropout)
        x = x.float().contiguous()
        e_t = e_t.float().contiguous()
        if quantize_denoised:
            pred_x0 = (x - s1 * e_t) / np.sqrt(a_t)
            pred_x0, _, _ = self.model.first_stage_model.quantize(pred_x0)
            x_prev = np.sqrt(a_prev) * pred_x0 + np.sqrt(1. - a_prev - sigma ** 2) * e_t + sigma * noise
            return x_prev, pred_x0
        return torch.ops.encdiff.ddim_step(x, e_t, noise, a_t, a_prev, sigma, s1)

    # ------------------------------------------------------------ captured loops
    def _entry(self, kind, cond, img, total, log_every_t, injected):
        """Cache entry (static input / output buffers) of a captured loop.  ``injected``: the
        noise comes from a caller's normals_sequence table (else drawn inside the graph)."""
        injected = bool(injected and self.ddim_eta)
        key = (kind, tuple(img.shape), total, self._sched_key, tuple(cond.shape), cond.dtype, log_every_t,
               injected)
        st = self._graphs.get(key)
        if st is None:
            dev = img.device
            logs = [i for i in range(total) if (total - i - 1) % log_every_t == 0 or i == 0]
            st = dict(key=key, x=torch.empty_like(img), x2=torch.empty_like(img), px0=torch.empty_like(img),
                      cond=torch.empty_like(cond), logs=logs,
                      log_x=torch.empty(len(logs), *img.shape, device=dev),
                      log_px0=torch.empty(len(logs), *img.shape, device=dev),
                      noise=torch.zeros((total if injected else 1), *img.shape, device=dev),
                      draw=bool(self.ddim_eta) and not injected, graph=None)
            self._graphs[key] = st
        st["cond"].copy_(cond)
        st["x"].copy_(img)
        return st

    def _fill_noise(self, st, normals_sequence, total):
        if self.ddim_eta and normals_sequence is not None:  # injected table (else: in-graph draws)
            st["noise"].copy_(normals_sequence[:total])

    def _refresh(self):
        f = getattr(self.model, "refresh_hip_weights", None)
        if f is not None:
            f()

    def _loop_graph(self, cond, img, total, log_every_t, intermediates, normals_sequence):
        """The whole loop as one HIP graph (unrolled: step i's coefficients and timestep are
        kernel arguments / a static timestep row)."""
        st = self._entry("loop", cond, img, total, log_every_t, normals_sequence is not None)
        self._fill_noise(st, normals_sequence, total)
        self._refresh()
        if st["graph"] is None:
            b = img.shape[0]
            steps = np.flip(self.ddim_timesteps)
            st["ts"] = torch.tensor(np.repeat(np.asarray(steps, dtype=np.int64)[:, None], b, axis=1), device=img.device)
            st["ts_col"] = st["ts"][:, 0].contiguous()  # one timestep per loop step (the FiLM table)
            x0 = st["x"].clone()
            self._loop_body(st, total)  # warm-up: allocations, kernel attributes, GEMM plans
            st["x"].copy_(x0)
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    self._loop_body(st, total)
            torch.cuda.current_stream().wait_stream(s)
            st["graph"] = g
            st["x"].copy_(x0)
        st["graph"].replay()
        for j in range(len(st["logs"])):
            intermediates["x_inter"].append(st["log_x"][j].clone())
            intermediates["pred_x0"].append(st["log_px0"][j].clone())
        return st["out"].clone(), intermediates

    def _hip_executor(self):
        """The bf16 HIP UNet executor behind the model (None: another backbone / precision)."""
        um = getattr(getattr(self.model, "model", None), "diffusion_model", None)
        if um is None or not hasattr(um, "executor") or getattr(um, "hip_precision", "bf16") == "fp32":
            return None
        return um.executor()

    def _loop_body(self, st, total):
        x, xn = st["x"], st["x2"]
        logs = st["logs"]
        noise_n = st["noise"].shape[0]
        # the conditioning is fixed and every row shares t within the loop: the executor computes the
        # concept-token K / V once and the FiLM rows of all S steps in one pass at step 0
        # (UNetExecutor.samp_ts / samp_i); ENCDIFF_DDIM_HOIST=0 recomputes them every step
        ex = self._hip_executor() if HOIST else None
        if ex is not None:
            ex.samp_ts, ex.samp_i = st["ts_col"], None
        um = self._borrow(True)
        try:
            self._loop_steps(st, total, x, xn, logs, noise_n, ex)
        finally:
            if ex is not None:
                ex.samp_ts = ex.samp_i = None
            if um is not None:
                um.borrow_eps = False

    def _borrow(self, on):
        """Let the HIP UNet hand its eps buffer over without a copy: each loop step consumes e_t
        (ddim_step) before the next forward overwrites it.  Returns the UNet (None: another backbone)."""
        um = getattr(getattr(self.model, "model", None), "diffusion_model", None)
        if um is None or not hasattr(um, "executor"):
            return None
        um.borrow_eps = on
        return um

    def _loop_steps(self, st, total, x, xn, logs, noise_n, ex):
        for i in range(total):
            index = total - i - 1
            if ex is not None:
                ex.samp_i = i
            e_t = self.model.apply_model(x, st["ts"][i], st["cond"])
            a_t, a_prev = float(self.ddim_alphas[index]), float(self.ddim_alphas_prev[index])
            sigma, s1 = float(self.ddim_sigmas[index]), float(self.ddim_sqrt_one_minus_alphas[index])
            if st["draw"]:
                st["noise"][0].normal_()
            ops.ddim_step(x, e_t.float().contiguous(), st["noise"][i if noise_n > 1 else 0], a_t, a_prev, sigma, s1,
                          xn, st["px0"])
            x, xn = xn, x
            if i in logs:
                j = logs.index(i)
                st["log_x"][j].copy_(x)
                st["log_px0"][j].copy_(st["px0"])
        st["out"] = x

    def _step_graph(self, cond, img, total, log_every_t, intermediates, normals_sequence):
        """Loops longer than GRAPH_MAX_STEPS: one captured step (coefficients, timestep and
        noise row looked up at a device step index), replayed S times."""
        st = self._entry("step", cond, img, total, log_every_t, normals_sequence is not None)
        self._fill_noise(st, normals_sequence, total)
        self._refresh()
        b = img.shape[0]
        if st["graph"] is None:
            dev = img.device
            st.update(t=torch.empty(b, device=dev, dtype=torch.long), idx=torch.zeros(1, device=dev, dtype=torch.int32),
                      i=torch.zeros(1, device=dev, dtype=torch.long), zrow=torch.empty_like(img))
            x0 = st["x"].clone()
            st["idx"].fill_(total - 1)
            self._step_body(st)
            st["x"].copy_(x0)
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    self._step_body(st)
            torch.cuda.current_stream().wait_stream(s)
            st["graph"] = g
            st["x"].copy_(x0)
        st["idx"].fill_(total - 1)
        st["i"].zero_()
        for i in range(total):
            st["graph"].replay()
            if i in st["logs"]:
                intermediates["x_inter"].append(st["x"].clone())
                intermediates["pred_x0"].append(st["px0"].clone())
        return st["x"].clone(), intermediates

    def _step_body(self, st):
        idx = st["idx"]
        st["t"].copy_(self._ts.index_select(0, idx.long()).expand(st["t"].shape[0]))
        um = self._borrow(True)
        try:
            e_t = self.model.apply_model(st["x"], st["t"], st["cond"])
        finally:
            if um is not None:
                um.borrow_eps = False
        if st["noise"].shape[0] > 1:  # noise row of loop step i (device counter)
            st["zrow"].copy_(st["noise"].index_select(0, st["i"]).view_as(st["zrow"]))
            st["i"].add_(1)
            z = st["zrow"]
        else:
            z = st["noise"][0]
            if st["draw"]:
                z.normal_()
        ops.ddim_step_indexed(st["x"], e_t.float().contiguous(), z, self._coef, idx, st["x2"], st["px0"],
                              advance=True)
        st["x"].copy_(st["x2"])
