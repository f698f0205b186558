"""Generate golden fixtures by running the REFERENCE implementation on CPU.

Run here (in the build container, where /root/reference exists):
    python tools/gen_golden.py

It imports the reference's own modules from /root/reference (read-only) with
sys.modules stubs for packages that are absent in this image (omegaconf,
pytorch_lightning, torchvision, taming, main_val) -- none of the stubs touches
the arithmetic of the hot path.  Weights come from the deterministic recipe in
oracle/encdiff_oracle.py (name-seeded), inputs from fixed seeds.  Outputs are
written as small .npz/.json fixtures into tests/golden/.  Nothing under
/root/reference is copied; only input/output data is stored.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, 'tests', 'golden')
sys.path.insert(0, REPO)

from oracle import encdiff_oracle as O  # noqa: E402


def install_shims():
    # omegaconf.listconfig.ListConfig (openaimodel_enc.py:477)
    om = types.ModuleType('omegaconf'); lc = types.ModuleType('omegaconf.listconfig')

    class ListConfig(list):
        pass
    lc.ListConfig = ListConfig; om.listconfig = lc
    sys.modules['omegaconf'] = om; sys.modules['omegaconf.listconfig'] = lc

    # pytorch_lightning (ddpm_enc.py:12,20; autoencoder.py:2)
    pl = types.ModuleType('pytorch_lightning')

    class LightningModule(nn.Module):
        current_epoch = 0
        global_step = 0

        @property
        def device(self):
            for p in self.parameters():
                return p.device
            return torch.device('cpu')

        def log(self, *a, **k):
            pass

        def log_dict(self, *a, **k):
            pass
    pl.LightningModule = LightningModule
    ut = types.ModuleType('pytorch_lightning.utilities')
    dist = types.ModuleType('pytorch_lightning.utilities.distributed')
    dist.rank_zero_only = lambda f: f
    ut.distributed = dist; pl.utilities = ut
    sys.modules['pytorch_lightning'] = pl
    sys.modules['pytorch_lightning.utilities'] = ut
    sys.modules['pytorch_lightning.utilities.distributed'] = dist

    tv = types.ModuleType('torchvision'); tvu = types.ModuleType('torchvision.utils')
    tvu.make_grid = lambda *a, **k: None; tv.utils = tvu
    sys.modules['torchvision'] = tv; sys.modules['torchvision.utils'] = tvu

    mv = types.ModuleType('main_val'); mv.eval_func = lambda *a, **k: {}
    sys.modules['main_val'] = mv

    # taming VectorQuantizer2 (autoencoder.py:11) -- state-dict-compatible stub,
    # never called by VQModelInterface.encode or by decode(force_not_quantize=True)
    tm = types.ModuleType('taming'); tmm = types.ModuleType('taming.modules')
    tmv = types.ModuleType('taming.modules.vqvae'); tmq = types.ModuleType('taming.modules.vqvae.quantize')

    class VectorQuantizer2(nn.Module):
        def __init__(self, n_e, e_dim, beta=0.25, remap=None, sane_index_shape=False, **kw):
            super().__init__()
            self.embedding = nn.Embedding(n_e, e_dim)
    tmq.VectorQuantizer2 = VectorQuantizer2
    for name, mod in (('taming', tm), ('taming.modules', tmm), ('taming.modules.vqvae', tmv),
                      ('taming.modules.vqvae.quantize', tmq)):
        sys.modules[name] = mod
    sys.path.insert(0, REF)


def load_yaml_cfg():
    import yaml
    with open(os.path.join(REF, 'configs/latent-diffusion/shapes3d-vq-4-16-encdiff.yaml')) as f:
        return yaml.safe_load(f)


class AttrDict(dict):
    __getattr__ = dict.__getitem__


def to_attr(d):
    if isinstance(d, dict):
        return AttrDict({k: to_attr(v) for k, v in d.items()})
    return d


def set_recipe(module: nn.Module, prefix: str, seed=0):
    """Overwrite every float parameter with the oracle's name-seeded recipe."""
    with torch.no_grad():
        for n, p in module.named_parameters():
            p.copy_(O.recipe_tensor(prefix + n, tuple(p.shape), seed))


def ddim_long(ldm, cond, S=200):
    """DDIM at the reference's log_images workload length (ddpm_enc.py:1474: ddim_steps=200,
    ddim_eta=1.), B = 2, eta in {0, 1}; the eta = 1 noise stream is torch.manual_seed(1234)
    then one CPU torch.randn(x.shape) per step (ddim.py:201 noise_like), as tests/test_gpu_ldm.py
    regenerates it.  Also the logged intermediates (log_every_t = 100 -> S/100 + 1 entries)."""
    from ldm.models.diffusion.ddim import DDIMSampler
    DDIMSampler.register_buffer = lambda self, name, attr: setattr(self, name, attr)
    res = {}
    for eta in (0.0, 1.0):
        sampler = DDIMSampler(ldm)
        xT = torch.randn(2, 3, 16, 16, generator=torch.Generator().manual_seed(5))
        torch.manual_seed(1234)
        with torch.no_grad():
            samples, inter = sampler.sample(S, 2, (3, 16, 16), cond[:2], eta=eta, verbose=False, x_T=xT)
        res['xT'] = xT.numpy()
        res[f'samples_eta{int(eta)}'] = samples.numpy()
        res[f'x_inter_eta{int(eta)}'] = torch.stack(inter['x_inter']).numpy()
        res[f'pred_x0_eta{int(eta)}'] = torch.stack(inter['pred_x0']).numpy()
    res['cond'] = cond[:2].numpy()
    res['S'] = np.array(S)
    np.savez_compressed(os.path.join(OUT, f'ddim_s{S}.npz'), **res)
    print(f'ddim S={S} written')


def main():
    only_ddim_long = '--only-ddim-long' in sys.argv
    install_shims()
    torch.set_num_threads(8)
    os.makedirs(OUT, exist_ok=True)
    from ldm.modules.diffusionmodules.openaimodel_enc import UNetModel, Encoder4
    from ldm.models.diffusion.ddim import DDIMSampler
    from ldm.modules.ema import LitEma
    from ldm.lr_scheduler import LambdaLinearScheduler
    from ldm.modules.diffusionmodules import util as U

    cfg = load_yaml_cfg()
    up = cfg['model']['params']['unet_config']['params']

    if only_ddim_long:
        return ddim_only(cfg)
    # ---------------- full UNet fwd + bwd, B=4 --------------------------------
    unet = UNetModel(**up)
    set_recipe(unet, '')
    unet.eval()
    g = torch.Generator().manual_seed(7)
    B = 4
    x = torch.randn(B, 3, 16, 16, generator=g).requires_grad_(True)
    t = torch.tensor([0, 10, 500, 999])
    ctx = (0.5 * torch.randn(B, 320, generator=g)).requires_grad_(True)
    gout = torch.randn(B, 3, 16, 16, generator=g)
    out = unet(x, t, context=[ctx])
    out.backward(gout)
    grad_names = ['time_embed.0.bias', 'time_embed.2.weight', 'input_blocks.0.0.weight',
                  'input_blocks.1.0.in_layers.0.weight', 'input_blocks.1.0.emb_layers.1.bias',
                  'input_blocks.1.1.transformer_blocks.0.attn1.to_q.weight',
                  'input_blocks.4.0.skip_connection.weight',
                  'input_blocks.7.1.transformer_blocks.0.attn2.to_v.weight',
                  'middle_block.1.transformer_blocks.0.attn2.to_k.weight',
                  'middle_block.1.norm.weight', 'output_blocks.5.2.out_layers.0.bias',
                  'output_blocks.11.1.proj_out.weight', 'output_blocks.11.1.transformer_blocks.0.ff.net.2.bias',
                  'out.0.weight', 'out.2.weight', 'out.2.bias']
    pd = dict(unet.named_parameters())
    fx = dict(x=x.detach().numpy(), t=t.numpy(), ctx=ctx.detach().numpy(), gout=gout.numpy(),
              eps=out.detach().numpy(), dx=x.grad.numpy(), dctx=ctx.grad.numpy())
    for n in grad_names:
        fx['grad.' + n] = pd[n].grad.numpy()
    np.savez_compressed(os.path.join(OUT, 'unet_b4.npz'), **fx)
    json.dump({k: list(v.shape) for k, v in unet.state_dict().items()},
              open(os.path.join(OUT, 'unet_state_dict_shapes.json'), 'w'), indent=0)
    print('unet eps std', out.std().item())

    # ---------------- Encoder4 (as-is cond stage) -----------------------------
    cp = cfg['model']['params']['cond_stage_config']['params']
    enc = Encoder4(**cp)
    set_recipe(enc, 'cond.')
    enc.train()
    img = torch.rand(4, 3, 64, 64, generator=g) * 2 - 1
    c = enc(img)
    enc.eval()
    u = enc.encoding(img)
    np.savez_compressed(os.path.join(OUT, 'encoder4.npz'), img=img.numpy(), c_train=c.detach().numpy(),
                        u_eval=u.detach().numpy())

    # ---------------- schedules ----------------------------------------------
    from ldm.models.diffusion.ddpm_enc import LatentDiffusion
    mp = to_attr(cfg['model']['params'])
    mp = AttrDict(dict(mp))
    fsc = to_attr(json.loads(json.dumps(cfg['model']['params']['first_stage_config'])))
    fsc['params'].pop('ckpt_path', None)
    kwargs = {k: v for k, v in cfg['model']['params'].items()
              if k not in ('first_stage_config', 'cond_stage_config', 'unet_config', 'scheduler_config',
                           'eval_name', 'monitor')}
    ldm = LatentDiffusion(first_stage_config=fsc, cond_stage_config=cfg['model']['params']['cond_stage_config'],
                          unet_config=cfg['model']['params']['unet_config'], **kwargs)
    sd_shapes = {k: list(v.shape) for k, v in ldm.state_dict().items()}
    json.dump(sd_shapes, open(os.path.join(OUT, 'latent_diffusion_state_dict_shapes.json'), 'w'), indent=0)
    sch = {k: getattr(ldm, k).numpy() for k in
           ['betas', 'alphas_cumprod', 'alphas_cumprod_prev', 'alphas_cumprod_next', 'sqrt_alphas_cumprod',
            'sqrt_one_minus_alphas_cumprod', 'log_one_minus_alphas_cumprod', 'sqrt_recip_alphas_cumprod',
            'sqrt_recipm1_alphas_cumprod', 'posterior_variance', 'posterior_log_variance_clipped',
            'posterior_mean_coef1', 'posterior_mean_coef2', 'lvlb_weights']}
    for S in (10, 50, 200):
        for eta in (0.0, 1.0):
            sig, a, ap, an = U.make_ddim_sampling_parameters(ldm.alphas_cumprod.cpu(),
                                                            U.make_ddim_timesteps('uniform', S, 1000, False),
                                                            eta, False)
            sch[f'ddim{S}_eta{int(eta)}_sigmas'] = np.asarray(sig, dtype=np.float64)
            sch[f'ddim{S}_eta{int(eta)}_alphas'] = np.asarray(a, dtype=np.float64)
            sch[f'ddim{S}_eta{int(eta)}_alphas_prev'] = np.asarray(ap, dtype=np.float64)
        sch[f'ddim{S}_timesteps'] = U.make_ddim_timesteps('uniform', S, 1000, False)
    np.savez_compressed(os.path.join(OUT, 'schedule.npz'), **sch)

    # ---------------- p_losses / apply_model through LatentDiffusion ---------
    set_recipe(ldm.model.diffusion_model, '')
    set_recipe(ldm.cond_stage_model, 'cond.')
    set_recipe(ldm.first_stage_model, 'vq.')
    ldm.eval()  # 'val' prefix; numerics identical
    g = torch.Generator().manual_seed(11)
    x0 = torch.randn(4, 3, 16, 16, generator=g)
    img = torch.rand(4, 3, 64, 64, generator=g) * 2 - 1
    tt = torch.tensor([3, 250, 640, 998])
    noise = torch.randn(4, 3, 16, 16, generator=g)
    torch.Tensor.cuda = lambda self, *a, **k: self  # ddpm_enc.py:1200 hard .cuda()
    with torch.no_grad():
        ldm.cond_stage_model.train()
        cond = ldm.get_learned_conditioning(img)
        loss, ld = ldm.p_losses(x0, cond, tt, noise=noise)
        z = ldm.encode_first_stage(img)
        ld_eps = ldm.apply_model(O.q_sample(O.sched_fp32(O.register_schedule()), x0, tt, noise), tt, cond)
    np.savez_compressed(os.path.join(OUT, 'p_losses.npz'), x0=x0.numpy(), img=img.numpy(), t=tt.numpy(),
                        noise=noise.numpy(), cond=cond.numpy(), loss=loss.numpy(),
                        loss_simple=ld['val/loss_simple'].numpy(), loss_vlb=ld['val/loss_vlb'].numpy(),
                        eps=ld_eps.numpy(), vq_z=z.numpy())

    # ---------------- DDIM sampling -----------------------------------------
    DDIMSampler.register_buffer = lambda self, name, attr: setattr(self, name, attr)
    res = {}
    for eta in (0.0, 1.0):
        sampler = DDIMSampler(ldm)
        xT = torch.randn(2, 3, 16, 16, generator=torch.Generator().manual_seed(5))
        torch.manual_seed(1234)
        with torch.no_grad():
            samples, inter = sampler.sample(10, 2, (3, 16, 16), cond[:2], eta=eta, verbose=False, x_T=xT)
        res[f'xT'] = xT.numpy()
        res[f'samples_eta{int(eta)}'] = samples.numpy()
        res[f'pred_x0_last_eta{int(eta)}'] = inter['pred_x0'][-1].numpy()
    res['cond'] = cond[:2].numpy()
    np.savez_compressed(os.path.join(OUT, 'ddim.npz'), **res)
    ddim_long(ldm, cond)

    # ---------------- EMA + AdamW + LR schedule -------------------------------
    small = nn.Sequential(nn.Linear(8, 16), nn.SiLU(), nn.Linear(16, 4))
    set_recipe(small, 'small.')
    ema = LitEma(small)
    opt = torch.optim.AdamW(small.parameters(), lr=1e-3)
    gg = torch.Generator().manual_seed(3)
    grads = []
    for step in range(3):
        opt.zero_grad()
        for p in small.parameters():
            gr = torch.randn(p.shape, generator=gg)
            p.grad = gr.clone()
            grads.append(gr.numpy())
        opt.step()
        ema(small)
    e = {'init.' + n: O.recipe_tensor('small.' + n, tuple(p.shape)).numpy() for n, p in small.named_parameters()}
    e.update({'param.' + n: p.detach().numpy() for n, p in small.named_parameters()})
    e.update({'ema.' + n: b.numpy() for n, b in ema.named_buffers()})
    e.update({f'grad{i}': gr for i, gr in enumerate(grads)})
    sched = LambdaLinearScheduler(warm_up_steps=[10000], cycle_lengths=[10000000000000], f_start=[1e-6],
                                  f_max=[1.], f_min=[1.])
    ns = np.array([0, 1, 5000, 9999, 10000, 20000, 37500])
    e['lr_n'] = ns
    e['lr_f'] = np.array([sched(int(n)) for n in ns], dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, 'ema_adamw_lr.npz'), **e)
    unet_bf16(cfg)
    print('fixtures written to', OUT)


def build_ldm(cfg):
    """The reference LatentDiffusion of the Shapes3D config with recipe weights (as main())."""
    from ldm.models.diffusion.ddpm_enc import LatentDiffusion
    fsc = to_attr(json.loads(json.dumps(cfg['model']['params']['first_stage_config'])))
    fsc['params'].pop('ckpt_path', None)
    kwargs = {k: v for k, v in cfg['model']['params'].items()
              if k not in ('first_stage_config', 'cond_stage_config', 'unet_config', 'scheduler_config',
                           'eval_name', 'monitor')}
    ldm = LatentDiffusion(first_stage_config=fsc, cond_stage_config=cfg['model']['params']['cond_stage_config'],
                          unet_config=cfg['model']['params']['unet_config'], **kwargs)
    set_recipe(ldm.model.diffusion_model, '')
    set_recipe(ldm.cond_stage_model, 'cond.')
    set_recipe(ldm.first_stage_model, 'vq.')
    ldm.eval()
    return ldm


def ddim_only(cfg):
    """--only-ddim-long: rebuild the p_losses conditioning exactly as main() does and write
    ddim_s200.npz only (the other fixtures untouched)."""
    ldm = build_ldm(cfg)
    g = torch.Generator().manual_seed(11)
    torch.randn(4, 3, 16, 16, generator=g)                 # x0 (same draw order as main())
    img = torch.rand(4, 3, 64, 64, generator=g) * 2 - 1
    torch.Tensor.cuda = lambda self, *a, **k: self
    with torch.no_grad():
        ldm.cond_stage_model.train()
        cond = ldm.get_learned_conditioning(img)
    ref = np.load(os.path.join(OUT, 'ddim.npz'))['cond']
    assert np.array_equal(cond[:2].numpy(), ref), 'conditioning differs from ddim.npz'
    ddim_long(ldm, cond)


def unet_bf16(cfg):
    """--only-bf16: the REFERENCE UNet on unet_b4.npz's inputs under torch.autocast(bf16) (CPU),
    forward and backward (the checkpoint recompute inside the backward autocast too), written as
    unet_b4_bf16.npz: eps, dx, dctx and the same 16 weight gradients.  This is the error the
    reference itself makes when it computes in bf16 -- the yardstick for the bf16 product
    backward's tolerance (tests/test_gpu_unet.py)."""
    from ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    up = cfg['model']['params']['unet_config']['params']
    unet = UNetModel(**up)
    set_recipe(unet, '')
    unet.eval()
    fx = np.load(os.path.join(OUT, 'unet_b4.npz'))
    x = torch.tensor(fx['x']).requires_grad_(True)
    ctx = torch.tensor(fx['ctx']).requires_grad_(True)
    with torch.autocast('cpu', dtype=torch.bfloat16):
        out = unet(x, torch.tensor(fx['t']), context=[ctx])
    # a second autocast region: the first one's cache of bf16 weight casts (made under the
    # checkpoint's no_grad forward) would cut the recompute off from the fp32 parameters
    with torch.autocast('cpu', dtype=torch.bfloat16):
        out.float().backward(torch.tensor(fx['gout']))
    pd = dict(unet.named_parameters())
    res = dict(eps=out.detach().float().numpy(), dx=x.grad.numpy(), dctx=ctx.grad.numpy())
    for k in fx.files:
        if k.startswith('grad.'):
            res[k] = pd[k[5:]].grad.float().numpy()
    np.savez_compressed(os.path.join(OUT, 'unet_b4_bf16.npz'), **res)
    print('unet_b4_bf16 written')


if __name__ == '__main__':
    if '--only-bf16' in sys.argv:
        install_shims()
        torch.set_num_threads(8)
        unet_bf16(load_yaml_cfg())
    else:
        main()
