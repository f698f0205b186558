"""The benchmarked training step itself, pinned to the oracle.

bench.py times HipTrainer at configs[1] (Shapes3D, B = 128 per GPU, the whole step captured
as one HIP graph).  This test runs exactly that object -- same batch size, same graph, the
B >= 64 code paths (GroupNorm statistics from the producing GEMMs, LayerNorm in GEMM
epilogues, the measured B = 128 tile / split-K plans, the fused AdamW + EMA + repack, the HIP
VQ encoder and Encoder4 trunk) -- with recipe weights (every layer non-zero, so eps and all
gradients carry data), and feeds each replay's image batch, timesteps and noise through
HipTrainer.enable_feed().  The CPU oracle (OracleTrainer, fp32, VQ encode included) starts
from the trainer's state after its eager warm-up steps and runs the same inputs.

Reference: ddpm_enc.py:360-375 (training_step), :773-844 (get_input), :1040-1053 (forward),
:1183-1253 (p_losses), :1598-1639 (AdamW), ema.py:25-44 (LitEma).

Tolerances (bf16 activations vs the fp32 reference): eps rel-L2 <= 3e-2 and
max-abs <= 6e-2; loss rel <= 1e-2; gradients rel-L2 <= 5e-2; AdamW / EMA parameter updates
rel-L2 <= 5e-2.  The L1 gradient seed sign(eps - noise)/N is discontinuous, so the oracle
back-propagates the seed the device computed (derived from the device eps) -- the loss value
itself is compared separately.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 128
LR = 1e-4
GRAD_NAMES = [  # UNet: every block type, the producer-statistics GroupNorms and LN epilogues
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
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def rig():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer
    from oracle import encdiff_oracle as O
    torch.set_num_threads(min(16, torch.get_num_threads()))
    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d"))
    with torch.no_grad():
        for n, p in ldm.model.diffusion_model.named_parameters():
            p.copy_(O.recipe_tensor(n, tuple(p.shape)))
        for n, p in ldm.cond_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("cond." + n, tuple(p.shape)))
        for n, p in ldm.first_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("vq." + n, tuple(p.shape)))
    ldm = ldm.cuda()
    # constant lr (the recipe's LambdaLinearScheduler starts at 1e-6 x lr, which would make
    # the AdamW update numerically empty); lr = B * base_lr as main_val.py:834-838
    ldm.use_scheduler = False
    tr = HipTrainer(ldm, B, base_lr=LR / B, graph=True, pool_size=2 * B)
    feed = tr.enable_feed()
    g = torch.Generator().manual_seed(2024)

    def inputs():
        u8 = torch.randint(0, 256, (B, 64, 64, 3), generator=g, dtype=torch.uint8)
        img = O.images_to_input(u8, torch.arange(B))
        return img, torch.randint(0, 1000, (B,), generator=g), torch.randn(B, 3, 16, 16, generator=g)

    img, t, noise = inputs()
    feed["img"].copy_(img); feed["t"].copy_(t); feed["noise"].copy_(noise)
    tr.init_scale_factor()
    sf_hip = float(ldm.scale_factor)
    tr.capture(warmup=2)  # two eager steps, then the graph the benchmark replays
    torch.cuda.synchronize()
    # the oracle starts from the trainer's state after the warm-up
    a = tr.arena
    unet_names = [n for n, _ in O.param_shapes(O.build_plan()).items()]
    cond_names = [n for n in O.encoder4_shapes() if "running" not in n and "num_batches" not in n]
    view = lambda buf, n: a.view_in(buf, n).detach().cpu().clone()  # noqa: E731
    unet = {n: view(a.master, n) for n in unet_names}
    cond = {n: view(a.master, "cond_stage_model." + n) for n in cond_names}
    m = {n: view(a.exp_avg, n) for n in unet_names}
    v = {n: view(a.exp_avg_sq, n) for n in unet_names}
    m.update({"cond." + n: view(a.exp_avg, "cond_stage_model." + n) for n in cond_names})
    v.update({"cond." + n: view(a.exp_avg_sq, "cond_stage_model." + n) for n in cond_names})
    ema = {n: view(a.ema, n) for n in unet_names}
    orc = O.OracleTrainer(O.build_plan(), lr=LR, vq=True)
    orc.load_state(unet, cond, m, v, tr.opt.step_count, ema, int(ldm.model_ema.num_updates))
    # scale_by_std (ddpm_enc.py:586-608) on the oracle's own fp32 latents of the first batch
    with torch.no_grad():
        orc.scale_factor = float(1.0 / O.vq_encode(orc.V, img).flatten().std())
    return dict(ldm=ldm, tr=tr, feed=feed, inputs=inputs, orc=orc, O=O, unet_names=unet_names,
                cond_names=cond_names, sf_hip=sf_hip)


def test_scale_factor(rig):
    r = rel(rig["sf_hip"], rig["orc"].scale_factor)
    print("scale_factor", rig["sf_hip"], rig["orc"].scale_factor, r)
    assert r < 1e-2


@pytest.mark.parametrize("step", [0, 1])
def test_graph_step_b128_matches_oracle(rig, step):
    tr, orc, feed, O = rig["tr"], rig["orc"], rig["feed"], rig["O"]
    a = tr.arena
    img, t, noise = rig["inputs"]()
    feed["img"].copy_(img); feed["t"].copy_(t); feed["noise"].copy_(noise)
    names = rig["unet_names"]
    before = {n: a.view_in(a.master, n).detach().cpu().clone() for n in names}
    ema_before = {n: a.view_in(a.ema, n).detach().cpu().clone() for n in names}
    cond_before = {n: a.view_in(a.master, "cond_stage_model." + n).detach().cpu().clone() for n in rig["cond_names"]}
    tr.step()  # graph replay: the benchmarked step
    torch.cuda.synchronize()
    eps = tr.unet._ex.eps.detach().cpu().clone()
    loss = tr.loss()
    seed = torch.sign(eps - noise) / eps.numel()
    o_before = {n: p.detach().clone() for n, p in orc.P.items()}
    lo = float(orc.step_images(img, t, noise, seed=seed))
    oeps = orc.last["eps"]
    # eps-prediction (rel-L2 <= 3e-2 and max-abs <= 6e-2)
    e_rel, e_max = rel(eps, oeps), (eps - oeps).abs().max().item()
    print(f"step {step}: eps rel-L2 {e_rel:.3e} max-abs {e_max:.3e} (|eps| max {oeps.abs().max():.2f}); "
          f"loss {loss:.5f} vs {lo:.5f}")
    assert e_rel < 3e-2 and e_max < 6e-2
    # the device loss is the L1 of the device eps (exact up to summation order) and the
    # reference's loss within the bf16 tolerance
    host = (eps.double() - noise.double()).abs().mean().item()
    assert abs(loss - host) / host < 1e-5, (loss, host)
    assert abs(loss - lo) / lo < 1e-2
    # weight gradients in the arena (UNet incl. producer-statistics GN / LN-epilogue layers; Encoder4)
    errs = {n: rel(a.view_in(a.grad, n), orc.P[n].grad) for n in GRAD_NAMES}
    errs.update({"cond." + n: rel(a.view_in(a.grad, "cond_stage_model." + n), orc.E[n].grad) for n in COND_NAMES})
    print(f"step {step}: grad rel-L2 " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    worst = max(errs.values())
    assert worst < 5e-2, max(errs, key=errs.get)
    # every UNet gradient at once
    gh = torch.cat([a.view_in(a.grad, n).detach().cpu().flatten() for n in names])
    go = torch.cat([orc.P[n].grad.flatten() for n in names])
    print(f"step {step}: worst listed grad rel-L2 {worst:.3e}; all UNet grads {rel(gh, go):.3e}")
    assert rel(gh, go) < 5e-2
    # AdamW update and EMA update (fp64 differences of fp32 values)
    dh = torch.cat([(a.view_in(a.master, n).detach().cpu().double() - before[n].double()).flatten() for n in names])
    do = torch.cat([(orc.P[n].detach().double() - o_before[n].double()).flatten() for n in names])
    eh = torch.cat([(a.view_in(a.ema, n).detach().cpu().double() - ema_before[n].double()).flatten() for n in names])
    eo = torch.cat([(orc.ema[n].double() - ema_before[n].double()).flatten() for n in names])
    ch = torch.cat([(a.view_in(a.master, "cond_stage_model." + n).detach().cpu().double()
                     - cond_before[n].double()).flatten() for n in rig["cond_names"]])
    co = torch.cat([(orc.E[n].detach().double() - cond_before[n].double()).flatten() for n in rig["cond_names"]])
    print(f"step {step}: AdamW update rel-L2 UNet {rel(dh, do):.3e} Encoder4 {rel(ch, co):.3e}; "
          f"EMA update {rel(eh, eo):.3e}")
    assert rel(dh, do) < 5e-2 and rel(ch, co) < 5e-2 and rel(eh, eo) < 5e-2
    # the two runs now differ by these updates only: carry the device state into the oracle
    # (the next step is compared from identical parameters again)
    with torch.no_grad():
        for n, p in orc.P.items():
            p.copy_(a.view_in(a.master, n).detach().cpu())
        for n in rig["cond_names"]:
            orc.E[n].copy_(a.view_in(a.master, "cond_stage_model." + n).detach().cpu())
        for n in names:
            orc.ema[n].copy_(a.view_in(a.ema, n).detach().cpu())
