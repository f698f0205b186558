"""Parity of the UNet executor on the wider, builder-defined UNet of BASELINE.json configs[4]
("CelebA 128x128 LDM, wider UNet + more concept tokens").

The reference has no config for it; the shapes follow SURVEY §8(d): VQ-f4 latent of a
128x128 image -> z (B,3,32,32), model_channels=128, latent_unit=40 concept tokens of
context_dim 16, otherwise the Shapes3D UNet family (openaimodel_enc.py:443-470).  Level-0
self-attention runs over S=1024 tokens (dh 16); the 512-channel levels have dh 64.

The CPU oracle (oracle/encdiff_oracle.py, pinned to the reference by the Shapes3D golden
fixtures) is the checker; its fp32 autograd gives the reference gradients.  The model runs
in bf16 on the GPU, so the tolerance is the north_star one used in test_gpu_unet.py:
eps rel-L2 <= 3e-2, gradients rel-L2 <= 5e-2.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

EPS_TOL = 3e-2
GRAD_TOL = 5e-2

WIDE_UNET = dict(image_size=32, in_channels=3, out_channels=3, model_channels=128,
                 attention_resolutions=[1, 2, 4], num_res_blocks=2,
                 channel_mult=[1, 2, 4, 4], num_heads=8, use_scale_shift_norm=True,
                 resblock_updown=True, use_spatial_transformer=True, context_dim=16,
                 latent_unit=40)

GRAD_KEYS = [
    "time_embed.0.bias", "input_blocks.0.0.weight", "input_blocks.1.0.in_layers.0.weight",
    "input_blocks.1.0.emb_layers.1.bias", "input_blocks.1.1.transformer_blocks.0.attn1.to_q.weight",
    "input_blocks.4.0.skip_connection.weight", "input_blocks.7.1.transformer_blocks.0.attn1.to_k.weight",
    "middle_block.1.transformer_blocks.0.attn2.to_k.weight", "middle_block.1.norm.weight",
    "output_blocks.5.2.out_layers.0.bias", "output_blocks.11.1.proj_out.weight",
    "output_blocks.11.1.transformer_blocks.0.ff.net.2.bias", "out.0.weight", "out.2.weight",
]


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def wide():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import encdiff_amd  # noqa: F401
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    from oracle import encdiff_oracle as O
    plan = O.build_plan(WIDE_UNET)
    P = O.recipe_params(O.param_shapes(plan))
    m = UNetModel(**WIDE_UNET)
    m.load_state_dict(P, strict=True)
    return m.cuda(), plan, P


def test_wide_unet_fwd_bwd_matches_oracle(wide):
    from oracle import encdiff_oracle as O
    m, plan, P = wide
    torch.manual_seed(31)
    B = 2
    x = torch.randn(B, 3, 32, 32)
    t = torch.tensor([3, 871])
    ctx = torch.randn(B, 40 * 16) * 0.5
    gout = torch.randn(B, 3, 32, 32)
    Pg = {k: v.clone().requires_grad_(k in GRAD_KEYS) for k, v in P.items()}
    ctx_ref = ctx.clone().requires_grad_(True)
    ref = O.unet_forward(Pg, plan, x, t, [ctx_ref])
    ref.backward(gout)

    m.executor()
    m._arena.zero_grad()
    ctx_d = ctx.cuda().requires_grad_(True)
    eps = m(x.cuda(), t.cuda(), context=[ctx_d])
    e = rel(eps.detach(), ref.detach())
    print("wide eps rel-L2 vs oracle:", e)
    assert e < EPS_TOL
    eps.backward(gout.cuda())
    d = rel(ctx_d.grad, ctx_ref.grad)
    print("wide d(context) rel-L2:", d)
    assert d < GRAD_TOL
    named = dict(m.named_parameters())
    for k in GRAD_KEYS:
        r = rel(named[k].grad, Pg[k].grad)
        print(k, r)
        assert r < GRAD_TOL, k


def test_wide_unet_batch_consistency(wide):
    """Training batch sizes switch on the producer-statistics GroupNorm and the training GEMM
    plans; image i's eps and d(context) at B=64 must match its own B=1 run (oracle-pinned
    path above) up to bf16 rounding: the GEMM tile / split-K plan differs per batch size, so
    the summation order (and each bf16 rounding after it) differs; bound = the tolerances."""
    m, _, _ = wide
    torch.manual_seed(8)
    B, i = 64, 37
    x = torch.randn(B, 3, 32, 32, device="cuda")
    t = torch.randint(0, 1000, (B,), device="cuda")
    c = torch.randn(B, 640, device="cuda")
    g = torch.randn(B, 3, 32, 32, device="cuda")
    cf = c.clone().requires_grad_(True)
    full = m(x, t, [cf])
    full.backward(g)
    c1 = c[i:i + 1].clone().requires_grad_(True)
    one = m(x[i:i + 1], t[i:i + 1], [c1])
    one.backward(g[i:i + 1])
    e = rel(one.detach(), full.detach()[i:i + 1])
    d = rel(c1.grad, cf.grad[i:i + 1])
    print("B=64 vs B=1 eps", e, "dctx", d)
    assert e < EPS_TOL and d < GRAD_TOL
