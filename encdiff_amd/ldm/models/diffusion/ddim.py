"""DDIMSampler -- mirror of ldm/models/diffusion/ddim.py:11-207 on the HIP path.

Same schedule construction (make_schedule, :24-54), same sampling loop order and
RNG consumption (one torch.randn of x's shape per step, :201), same update
(p_sample_ddim, :188-207) -- the update itself is one HIP kernel.  With
``use_graph=True`` (default on a HIP device, when no per-step callbacks, masks or
guidance are requested) one step -- UNet forward + DDIM update -- is captured into
a HIP graph whose coefficients and timestep are looked up from device tables at a
device step index, and the graph is replayed S times.
"""
from __future__ import annotations

import numpy as np
import torch

from encdiff_amd import ops
from ...modules.diffusionmodules.util import make_ddim_sampling_parameters, make_ddim_timesteps, noise_like


class DDIMSampler(object):
    def __init__(self, model, schedule="linear", use_graph=True, **kwargs):
        super().__init__()
        self.model = model
        self.ddpm_num_timesteps = model.num_timesteps
        self.schedule = schedule
        self.use_graph = use_graph
        self._graphs = {}

    def register_buffer(self, name, attr):
        if isinstance(attr, torch.Tensor):
            attr = attr.to(self.model.device)
        setattr(self, name, attr)

    def make_schedule(self, ddim_num_steps, ddim_discretize="uniform", ddim_eta=0., verbose=True):
        self.ddim_timesteps = make_ddim_timesteps(ddim_discretize, ddim_num_steps, self.ddpm_num_timesteps,
                                                  verbose=verbose)
        alphas_cumprod = self.model.alphas_cumprod
        assert alphas_cumprod.shape[0] == self.ddpm_num_timesteps
        to_t = lambda x: x.clone().detach().to(torch.float32).to(self.model.device)
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
        # device tables for the captured step: coef[index] = (a_t, a_prev, sigma, sqrt(1-a_t)); ts[index]
        coef = np.stack([a, ap, sig, self.ddim_sqrt_one_minus_alphas], axis=1).astype(np.float32)
        self._coef = torch.tensor(coef, device=self.model.device)
        self._ts = torch.tensor(np.asarray(self.ddim_timesteps, dtype=np.int64), device=self.model.device)

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
                                  unconditional_conditioning=unconditional_conditioning)

    @torch.no_grad()
    def ddim_sampling(self, cond, shape, x_T=None, ddim_use_original_steps=False, callback=None, timesteps=None,
                      quantize_denoised=False, mask=None, x0=None, img_callback=None, log_every_t=100,
                      temperature=1., noise_dropout=0., score_corrector=None, corrector_kwargs=None,
                      unconditional_guidance_scale=1., unconditional_conditioning=None):
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
        intermediates = {"x_inter": [img], "pred_x0": [img]}
        simple = (callback is None and img_callback is None and mask is None and not quantize_denoised and
                  noise_dropout == 0. and score_corrector is None and temperature == 1. and
                  (unconditional_conditioning is None or unconditional_guidance_scale == 1.))
        if self.use_graph and simple and img.is_cuda and timesteps is None:
            return self._graph_sampling(cond, img, total, log_every_t, intermediates)
        for i, step in enumerate(np.flip(steps)):
            index = total - i - 1
            ts = torch.full((b,), int(step), device=device, dtype=torch.long)
            if mask is not None:
                img = self.model.q_sample(x0, ts) * mask + (1. - mask) * img
            img, pred_x0 = self.p_sample_ddim(img, cond, ts, index=index, quantize_denoised=quantize_denoised,
                                              temperature=temperature, noise_dropout=noise_dropout,
                                              score_corrector=score_corrector, corrector_kwargs=corrector_kwargs,
                                              unconditional_guidance_scale=unconditional_guidance_scale,
                                              unconditional_conditioning=unconditional_conditioning)
            if callback:
                callback(i)
            if img_callback:
                img_callback(pred_x0, i)
            if index % log_every_t == 0 or index == total - 1:
                intermediates["x_inter"].append(img)
                intermediates["pred_x0"].append(pred_x0)
        return img, intermediates

    @torch.no_grad()
    def p_sample_ddim(self, x, c, t, index, repeat_noise=False, use_original_steps=False, quantize_denoised=False,
                      temperature=1., noise_dropout=0., score_corrector=None, corrector_kwargs=None,
                      unconditional_guidance_scale=1., unconditional_conditioning=None):
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
        noise = noise_like(x.shape, x.device, repeat_noise) * temperature
        if noise_dropout > 0.:
            noise = torch.nn.functional.dropout(noise, p=noise_dropout)
        x = x.float().contiguous()
        e_t = e_t.float().contiguous()
        x_prev = torch.empty_like(x)
        pred_x0 = torch.empty_like(x)
        if quantize_denoised:
            pred_x0 = (x - s1 * e_t) / np.sqrt(a_t)
            pred_x0, _, _ = self.model.first_stage_model.quantize(pred_x0)
            x_prev = np.sqrt(a_prev) * pred_x0 + np.sqrt(1. - a_prev - sigma ** 2) * e_t + sigma * noise
            return x_prev, pred_x0
        ops.ddim_step(x, e_t, noise.contiguous(), a_t, a_prev, sigma, s1, x_prev, pred_x0)
        return x_prev, pred_x0

    # ------------------------------------------------------------ captured loop
    def _graph_sampling(self, cond, img, total, log_every_t, intermediates):
        dev = img.device
        b = img.shape[0]
        key = (tuple(img.shape), total, cond.data_ptr() if isinstance(cond, torch.Tensor) else id(cond))
        st = self._graphs.get(key)
        if st is None:
            st = dict(x=torch.empty_like(img), x_next=torch.empty_like(img), px0=torch.empty_like(img),
                      t=torch.empty(b, device=dev, dtype=torch.long), idx=torch.zeros(1, device=dev, dtype=torch.int32))
            st["idx"].fill_(total - 1)
            self._step_eager(st, cond)  # warm-up (allocations, kernel attributes)
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    self._step_eager(st, cond)
            torch.cuda.current_stream().wait_stream(s)
            st["graph"] = g
            self._graphs[key] = st
        st["x"].copy_(img)
        st["idx"].fill_(total - 1)
        for i in range(total):
            index = total - i - 1
            st["graph"].replay()
            if index % log_every_t == 0 or index == total - 1:
                intermediates["x_inter"].append(st["x"].clone())
                intermediates["pred_x0"].append(st["px0"].clone())
        return st["x"].clone(), intermediates

    def _step_eager(self, st, cond):
        idx = st["idx"]
        st["t"].copy_(self._ts.index_select(0, idx.long()).expand(st["t"].shape[0]))
        e_t = self.model.apply_model(st["x"], st["t"], cond)
        noise = torch.randn(st["x"].shape, device=st["x"].device)
        ops.ddim_step_indexed(st["x"], e_t, noise, self._coef, idx, st["x_next"], st["px0"], advance=True)
        st["x"].copy_(st["x_next"])
