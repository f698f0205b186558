"""The fp32 path through the C-ABI (SURVEY §8(b) convention 5; include/encdiff_hip.h `dtype`):
the GEMM, GroupNorm, LayerNorm, attention and elementwise entry points with ENCDIFF_DT_F32, and
the whole denoiser forward on them (encdiff_amd/unet_f32.py, UNetModel hip_precision="fp32")
held to the fp32 tolerance of SURVEY.md §8(c), 1e-4 rel-L2, against the REFERENCE's own output
(tests/golden/unet_b4.npz, tools/gen_golden.py: openaimodel_enc.py:712-748 on CPU, fp32).
Per-op checks against torch fp32 at 2e-5."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import encdiff_amd  # noqa: F401
    return torch.device("cuda")


@pytest.mark.parametrize("cin,cout,h,rs", [(64, 64, 16, 0), (8, 64, 16, 0), (128, 256, 4, 2), (192, 64, 16, 0)])
def test_conv3x3_f32(dev, cin, cout, h, rs):
    from encdiff_amd import _lib as L, ops
    from encdiff_amd.ops import Geom
    g = torch.Generator().manual_seed(cin + cout)
    B = 4
    hs = h // 2 if rs == L.RESAMPLE_UP2 else h
    x = torch.randn(B, cin, hs, hs, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    b = torch.randn(cout, generator=g)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if rs == L.RESAMPLE_UP2 else x
    ref = F.conv2d(xin.double(), w.double(), b.double(), padding=1)
    rows = x.permute(0, 2, 3, 1).reshape(-1, cin).contiguous().to(dev)
    wk = w.permute(0, 2, 3, 1).reshape(cout, 9 * cin).contiguous().to(dev)
    y = torch.empty(B * h * h, cout, device=dev)
    ops.conv3x3_f32(rows, Geom(B, h, h), cin, wk, y, bias=b.to(dev), resample=rs)
    got = y.cpu().view(B, h, h, cout).permute(0, 3, 1, 2)
    r = rel(got, ref)
    print("conv3x3 fp32", cin, cout, h, rs, r)
    assert r < 2e-6


def test_groupnorm_layernorm_f32(dev):
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    g = torch.Generator().manual_seed(5)
    B, C, H = 4, 128, 8
    x = torch.randn(B, C, H, H, generator=g) * 3 + 1
    gam, bet = torch.randn(C, generator=g), torch.randn(C, generator=g)
    film = torch.randn(B, 2 * C, generator=g) * 0.3
    ref = F.group_norm(x.double(), 32, gam.double(), bet.double(), 1e-5)
    ref = ref * (1 + film[:, :C, None, None].double()) + film[:, C:, None, None].double()
    ref = F.silu(ref)
    rows = x.permute(0, 2, 3, 1).reshape(-1, C).contiguous().to(dev)
    y = torch.empty_like(rows)
    st = torch.empty(B * 64, device=dev)
    ops.groupnorm_f32(rows, Geom(B, H, H), gam.to(dev), bet.to(dev), y, st, 1e-5, True, film=film.to(dev),
                      ld_film=2 * C)
    r = rel(y.cpu().view(B, H, H, C).permute(0, 3, 1, 2), ref)
    print("groupnorm fp32", r)
    assert r < 2e-6
    t = torch.randn(300, C, generator=g) * 2 - 0.5
    lref = F.layer_norm(t.double(), (C,), gam.double(), bet.double(), 1e-5)
    yt = torch.empty(300, C, device=dev)
    ops.layernorm_f32(t.to(dev), gam.to(dev), bet.to(dev), yt)
    r = rel(yt, lref)
    print("layernorm fp32", r)
    assert r < 2e-6


@pytest.mark.parametrize("sq,sk,dh", [(256, 256, 8), (64, 20, 16), (16, 20, 32), (200, 300, 64)])
def test_attention_f32(dev, sq, sk, dh):
    from encdiff_amd import ops
    g = torch.Generator().manual_seed(sq + dh)
    B, h = 2, 4
    q = torch.randn(B, sq, h * dh, generator=g)
    k = torch.randn(B, sk, h * dh, generator=g)
    v = torch.randn(B, sk, h * dh, generator=g)
    split = lambda t: t.view(B, -1, h, dh).permute(0, 2, 1, 3).double()  # noqa: E731
    ref = torch.softmax(split(q) @ split(k).transpose(-1, -2) * dh ** -0.5, -1) @ split(v)
    ref = ref.permute(0, 2, 1, 3).reshape(B * sq, h * dh)
    o = torch.empty(B * sq, h * dh, device=dev)
    ops.attention_f32(q.view(-1, h * dh).to(dev), k.view(-1, h * dh).to(dev), v.view(-1, h * dh).to(dev), o, B, h,
                      sq, sk, dh)
    r = rel(o, ref)
    print("attention fp32", sq, sk, dh, r)
    assert r < 2e-6


def test_unet_forward_fp32_matches_reference(dev, golden_dir):
    """UNetModel.forward at hip_precision='fp32' vs the reference's own eps (B = 4, recipe
    weights): rel-L2 <= 1e-4 (SURVEY.md §8(c) fp32 kernels)."""
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from oracle import encdiff_oracle as O
    fx = np.load(os.path.join(golden_dir, "unet_b4.npz"))
    ucfg = model_config("shapes3d")["params"]["unet_config"]
    unet = instantiate_from_config(ucfg)
    with torch.no_grad():
        for n, p in unet.named_parameters():
            p.copy_(O.recipe_tensor(n, tuple(p.shape)))
    unet = unet.to(dev).eval()
    x, t, ctx = (torch.tensor(fx[k]).to(dev) for k in ("x", "t", "ctx"))
    with torch.no_grad():
        bf = unet(x, t, context=[ctx]).cpu()
        unet.hip_precision = "fp32"
        e32 = unet(x, t, context=[ctx]).cpu()
        unet.hip_precision = "bf16"
    r32, rbf = rel(e32, fx["eps"]), rel(bf, fx["eps"])
    print(f"UNet B=4 vs reference: fp32 path rel-L2 {r32:.3e} max-abs {(e32 - torch.tensor(fx['eps'])).abs().max():.3e}; "
          f"bf16 product path {rbf:.3e}")
    assert r32 < 1e-4
    with pytest.raises(RuntimeError, match="forward-only"):
        unet.hip_precision = "fp32"
        try:
            unet(x, t, context=[ctx])
        finally:
            unet.hip_precision = "bf16"
