"""BASELINE.json configs[4] end to end: the builder-defined CelebA 128x128 LatentDiffusion
(encdiff_amd.configs.CELEBA128: VQ-f4 latent (B, 3, 32, 32), model_channels 128, 40 concept
tokens, Encoder4 with a fifth stride-2 stage, fp8 (e4m3) scores in the S = 1024 self-attention)
trained by the same graph-captured HipTrainer as the benchmark, vs the CPU oracle configured
alike (its fp8 scores emulated with torch.float8_e4m3fn).  No reference config exists for
this one, so the oracle -- pinned to the reference on Shapes3D -- is
the checker; tolerances as in test_gpu_trainer.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 8
LR = 1e-4


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_celeba128_step_matches_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer
    from oracle import encdiff_oracle as O
    torch.set_num_threads(min(16, torch.get_num_threads()))
    cfg = model_config("celeba128")
    ucfg = cfg["params"]["unet_config"]["params"]
    torch.manual_seed(0)
    ldm = instantiate_from_config(cfg)
    with torch.no_grad():
        for n, p in ldm.model.diffusion_model.named_parameters():
            p.copy_(O.recipe_tensor(n, tuple(p.shape)))
        for n, p in ldm.cond_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("cond." + n, tuple(p.shape)))
        for n, p in ldm.first_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("vq." + n, tuple(p.shape)))
    ldm = ldm.cuda()
    ldm.use_scheduler = False
    st = [t for t in ldm.model.diffusion_model._spec.sts if t.fp8]
    assert st and all(t.h == 32 for t in st), "fp8 scores on the 32x32 (S = 1024) level only"
    tr = HipTrainer(ldm, B, base_lr=LR / B, graph=True, pool_size=2 * B)
    assert tr.res == 128
    feed = tr.enable_feed()
    g = torch.Generator().manual_seed(77)

    def inputs():
        u8 = torch.randint(0, 256, (B, 128, 128, 3), generator=g, dtype=torch.uint8)
        return (O.images_to_input(u8, torch.arange(B)), torch.randint(0, 1000, (B,), generator=g),
                torch.randn(B, 3, 32, 32, generator=g))

    img, t, noise = inputs()
    feed["img"].copy_(img); feed["t"].copy_(t); feed["noise"].copy_(noise)
    tr.init_scale_factor()
    tr.capture(warmup=1)
    torch.cuda.synchronize()
    a = tr.arena
    plan = O.build_plan(ucfg)
    unet_names = list(O.param_shapes(plan))
    cond_names = [n for n in O.encoder4_shapes(latent_unit=40, image_size=128)
                  if "running" not in n and "num_batches" not in n]
    view = lambda buf, n: a.view_in(buf, n).detach().cpu().clone()  # noqa: E731
    orc = O.OracleTrainer(plan, lr=LR, vq=True, image_size=128)
    m = {n: view(a.exp_avg, n) for n in unet_names}
    v = {n: view(a.exp_avg_sq, n) for n in unet_names}
    m.update({"cond." + n: view(a.exp_avg, "cond_stage_model." + n) for n in cond_names})
    v.update({"cond." + n: view(a.exp_avg_sq, "cond_stage_model." + n) for n in cond_names})
    orc.load_state({n: view(a.master, n) for n in unet_names},
                   {n: view(a.master, "cond_stage_model." + n) for n in cond_names}, m, v, tr.opt.step_count,
                   {n: view(a.ema, n) for n in unet_names}, int(ldm.model_ema.num_updates))
    orc.scale_factor = float(ldm.scale_factor)
    img, t, noise = inputs()
    feed["img"].copy_(img); feed["t"].copy_(t); feed["noise"].copy_(noise)
    before = {n: view(a.master, n) for n in unet_names}
    tr.step()
    torch.cuda.synchronize()
    eps = tr.unet._ex.eps.detach().cpu().clone()
    loss = tr.loss()
    seed = torch.sign(eps - noise) / eps.numel()
    o_before = {n: p.detach().clone() for n, p in orc.P.items()}
    lo = float(orc.step_images(img, t, noise, seed=seed))
    oeps = orc.last["eps"]
    e_rel, e_max = rel(eps, oeps), (eps - oeps).abs().max().item()
    gh = torch.cat([a.view_in(a.grad, n).detach().cpu().flatten() for n in unet_names])
    go = torch.cat([orc.P[n].grad.flatten() for n in unet_names])
    ch = torch.cat([a.view_in(a.grad, "cond_stage_model." + n).detach().cpu().flatten() for n in cond_names])
    co = torch.cat([orc.E[n].grad.flatten() for n in cond_names])
    dh = torch.cat([(view(a.master, n).double() - before[n].double()).flatten() for n in unet_names])
    do = torch.cat([(orc.P[n].detach().double() - o_before[n].double()).flatten() for n in unet_names])
    print(f"configs[4] B={B}: eps rel-L2 {e_rel:.3e} max-abs {e_max:.3e}; loss {loss:.5f} vs {lo:.5f}; "
          f"UNet grads {rel(gh, go):.3e}; Encoder4 grads {rel(ch, co):.3e}; AdamW update {rel(dh, do):.3e}")
    worst = max(((rel(a.view_in(a.grad, n), orc.P[n].grad), n) for n in unet_names if orc.P[n].grad.norm() > 0))
    print("worst UNet parameter gradient", worst)
    assert e_rel < 3e-2 and e_max < 6e-2
    assert abs(loss - lo) / lo < 1e-2
    assert rel(gh, go) < 5e-2 and rel(ch, co) < 5e-2 and rel(dh, do) < 5e-2
    assert worst[0] < 5e-2, worst
