"""LatentDiffusion API on the HIP path vs the reference (fixtures) and the oracle.

Tolerances: loss values rel 1e-2; gradients rel-L2 5e-2; DDIM samples rel-L2 3e-2
(bf16 UNet activations vs fp32 reference).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def ldm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from oracle import encdiff_oracle as O
    m = instantiate_from_config(model_config("shapes3d"))
    with torch.no_grad():
        for n, p in m.model.diffusion_model.named_parameters():
            p.copy_(O.recipe_tensor(n, tuple(p.shape)))
        for n, p in m.cond_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("cond." + n, tuple(p.shape)))
        for n, p in m.first_stage_model.named_parameters():
            p.copy_(O.recipe_tensor("vq." + n, tuple(p.shape)))
    return m.cuda()


def test_p_losses_matches_reference(ldm, golden_dir):
    fx = np.load(os.path.join(golden_dir, "p_losses.npz"))
    ldm.eval()
    with torch.no_grad():
        cond = torch.tensor(fx["cond"]).cuda()
        loss, ld = ldm.p_losses(torch.tensor(fx["x0"]).cuda(), cond, torch.tensor(fx["t"]).cuda(),
                                noise=torch.tensor(fx["noise"]).cuda())
        z = ldm.encode_first_stage(torch.tensor(fx["img"]).cuda())
    print("loss", float(loss), float(fx["loss"]))
    assert abs(float(loss) - float(fx["loss"])) / abs(float(fx["loss"])) < 1e-2
    assert abs(float(ld["val/loss_vlb"]) - float(fx["loss_vlb"])) / abs(float(fx["loss_vlb"])) < 1e-2
    assert rel(z, fx["vq_z"]) < 1e-3  # as-is first stage (torch fp32 on the GPU)
    ldm.train()


def test_training_gradients_match_oracle(ldm):
    """Backward through UNet (HIP) and Encoder4 (torch): arena gradients vs the oracle's
    autograd gradients on identical (x0, img, t, noise).  Both sides get the SAME upstream
    seed (the L1 seed sign(eps_hat - eps) is discontinuous, so a bf16/fp32 eps difference
    would otherwise flip seed entries); the loss value itself is compared separately."""
    from oracle import encdiff_oracle as O
    ldm.train()
    ldm.setup_hip_training()
    torch.manual_seed(3)
    B = 8
    x0, img = torch.randn(B, 3, 16, 16), torch.rand(B, 3, 64, 64) * 2 - 1
    t, noise = torch.randint(0, 1000, (B,)), torch.randn(B, 3, 16, 16)
    ldm._arena.zero_grad()
    c = ldm.get_learned_conditioning(img.cuda())
    loss, _ = ldm.p_losses(x0.cuda(), c, t.cuda(), noise=noise.cuda())
    P = {k: v.requires_grad_(True) for k, v in O.recipe_params(O.param_shapes(O.build_plan())).items()}
    E = O.encoder4_params()
    E = {k: (v.requires_grad_(True) if v.is_floating_point() and "running" not in k else v) for k, v in E.items()}
    sched = O.sched_fp32(O.register_schedule())
    cr = O.encoder4_forward(E, img)
    out = O.unet_forward(P, O.build_plan(), O.q_sample(sched, x0, t, noise), t, [cr])
    lref, _ = O.p_losses_from_output(sched, out, noise, t)
    assert abs(float(loss.detach()) - float(lref.detach())) / float(lref) < 1e-2
    # shared upstream gradient for the model outputs
    seed = torch.sign(out.detach() - noise) / out.numel()
    ldm._arena.zero_grad()
    c = ldm.get_learned_conditioning(img.cuda())
    eps = ldm.apply_model(ldm.q_sample(x0.cuda(), t.cuda(), noise.cuda()), t.cuda(), c)
    eps.backward(seed.cuda())
    out.backward(seed)
    unet = dict(ldm.model.diffusion_model.named_parameters())
    for n in ["time_embed.0.weight", "input_blocks.1.0.in_layers.2.weight", "middle_block.1.proj_in.weight",
              "output_blocks.8.2.out_layers.3.weight", "out.2.weight", "output_blocks.3.1.norm.bias"]:
        r = rel(unet[n].grad, P[n].grad)
        print(n, r)
        assert r < 5e-2, n
    # Encoder4's trunk runs in bf16 with ReLU masks: near-zero pre-activations flip (see
    # test_encoder4_trunk_hip), hence the looser bound on its first conv
    cond = dict(ldm.cond_stage_model.named_parameters())
    for n, tol in [("encoder.0.weight", 0.2), ("encoder.16.weight", 5e-2), ("net.3.4.weight", 5e-2)]:
        r = rel(cond[n].grad, E[n].grad)
        print("cond", n, r)
        assert r < tol, n


@pytest.mark.parametrize("graph", [False, True])
def test_ddim_matches_reference(ldm, golden_dir, graph):
    from encdiff_amd.ldm.models.diffusion.ddim import DDIMSampler
    fx = np.load(os.path.join(golden_dir, "ddim.npz"))
    cond = torch.tensor(fx["cond"]).cuda()
    s = DDIMSampler(ldm, use_graph=graph)
    with torch.no_grad():
        out, inter = s.sample(10, 2, (3, 16, 16), cond, eta=0.0, verbose=False, x_T=torch.tensor(fx["xT"]).cuda())
    r = rel(out, fx["samples_eta0"])
    print("ddim eta0 graph=%s rel-L2" % graph, r)
    assert r < 3e-2
    assert len(inter["x_inter"]) >= 2


def test_vq_encoder_hip():
    """HIP VQ first-stage encoder (bf16 NHWC kernels) vs the as-is fp32 torch encoder on
    the same (random-init) weights: quant_conv(encoder(x)) rel-L2 < 2e-2."""
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    fs = ldm.first_stage_model
    x = torch.rand(8, 3, 64, 64, device="cuda") * 2 - 1
    with torch.no_grad():
        ref = fs.encode(x)
        fs.enable_hip()
        out = fs.encode(x)
    assert out.shape == ref.shape
    err = ((out - ref).norm() / ref.norm()).item()
    assert err < 2e-2, err
    # in-place weight change (load_state_dict) is picked up
    with torch.no_grad():
        fs.encoder.conv_out.bias.add_(0.5)
        fs._hip_encoder.enc.conv_out.bias  # same module
        out2 = fs.encode(x)
        fs._hip_encoder = None
        ref2 = fs.encode(x)
    assert ((out2 - ref2).norm() / ref2.norm()).item() < 2e-2


def test_encoder4_trunk_hip():
    """HIP Encoder4 convolution trunk (bf16 NHWC GEMMs + BatchNorm kernels) vs the as-is fp32
    torch modules on the same weights, training mode: output u rel-L2 < 3e-2, trunk parameter
    gradients within the ReLU-mask bound below, BN running statistics updated alike."""
    import copy
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    torch.manual_seed(1)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    ldm.train()
    ref = copy.deepcopy(ldm.cond_stage_model)
    ldm.setup_hip_training()
    enc = ldm.cond_stage_model
    assert enc._trunk is not None, "trunk not bound to the arena"
    x = torch.rand(16, 3, 64, 64, device="cuda") * 2 - 1
    proj = torch.randn(16, enc.latent_unit, device="cuda")
    ldm._arena.zero_grad()
    u = enc.encoding(x)
    (u * proj).sum().backward()
    u_ref = ref.encoding(x)
    (u_ref * proj).sum().backward()
    r = rel(u.detach(), u_ref.detach())
    print("u rel-L2", r)
    assert r < 3e-2
    # ReLU masks are evaluated on bf16 activations: the ~1% of near-zero pre-activations whose
    # sign differs from the fp32 reference each pass a full upstream gradient, which shows as
    # ~10% rel-L2 on random-init gradients (the kernels themselves are pinned to 1e-2 in
    # test_gpu_ops.py).  Gradients must agree to 0.2 rel-L2 and cos > 0.98; conv biases that
    # feed a BatchNorm have zero true gradient: their bf16 residue is measured against the
    # following BN's beta gradient (same scale).
    got = dict(enc.named_parameters())
    pre_bn_bias = {"encoder.0.bias": "encoder.1.bias", "encoder.3.bias": "encoder.4.bias",
                   "encoder.6.bias": "encoder.7.bias", "encoder.8.bias": "encoder.9.bias",
                   "encoder.11.convs.1.bias": "encoder.11.convs.2.bias", "encoder.11.convs.4.bias": "encoder.12.bias",
                   "encoder.14.convs.1.bias": "encoder.14.convs.2.bias"}
    for n, p in ref.named_parameters():
        if not n.startswith("encoder."):
            continue
        g, gr = got[n].grad.double().flatten(), p.grad.double().flatten()
        if n in pre_bn_bias:
            scale = got[pre_bn_bias[n]].grad.double().norm()
            print(n, "residue", (g.norm() / scale).item())
            assert g.norm() < 0.1 * scale, n
            continue
        e, cos = rel(g, gr), torch.nn.functional.cosine_similarity(g, gr, dim=0).item()
        print(n, e, cos)
        assert e < 0.2 and cos > 0.98, n
    for (n, b), (_, b_ref) in zip(enc.named_buffers(), ref.named_buffers()):
        if "running" in n:
            assert rel(b, b_ref) < 2e-2, n
    # two identical steps give bitwise identical gradients (deterministic BN folds)
    g1 = ldm._arena.grad.clone()
    ldm._arena.zero_grad()
    u = enc.encoding(x)
    (u * proj).sum().backward()
    assert torch.equal(g1, ldm._arena.grad)
