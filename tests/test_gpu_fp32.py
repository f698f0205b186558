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


def test_unet_backward_fp32_matches_reference(dev, golden_dir):
    """The fp32 BACKWARD through the C-ABI (UNetModel hip_precision="fp32" with grad: unet_f32.py)
    vs the reference's own fp32 autograd on the fixture (tests/golden/unet_b4.npz,
    openaimodel_enc.py:712-748): d x_t, d context and all 16 fixture weight / bias gradients
    within 1e-4 rel-L2 each (SURVEY.md §8(c) fp32 tolerance)."""
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from oracle import encdiff_oracle as O
    fx = np.load(os.path.join(golden_dir, "unet_b4.npz"))
    ucfg = model_config("shapes3d")["params"]["unet_config"]
    unet = instantiate_from_config(ucfg)
    with torch.no_grad():
        for n, p in unet.named_parameters():
            p.copy_(O.recipe_tensor(n, tuple(p.shape)))
    unet = unet.to(dev)
    unet.hip_precision = "fp32"
    try:
        unet.executor()
        unet._arena.zero_grad()
        x = torch.tensor(fx["x"]).to(dev).requires_grad_(True)
        ctx = torch.tensor(fx["ctx"]).to(dev).requires_grad_(True)
        eps = unet(x, torch.tensor(fx["t"]).to(dev), context=[ctx])
        e = rel(eps.detach(), fx["eps"])
        eps.backward(torch.tensor(fx["gout"]).to(dev))
        torch.cuda.synchronize()
    finally:
        unet.hip_precision = "bf16"
    checks = {"dx": (x.grad, fx["dx"]), "dctx": (ctx.grad, fx["dctx"])}
    named = dict(unet.named_parameters())
    for k in fx.files:
        if k.startswith("grad."):
            checks[k[5:]] = (named[k[5:]].grad, fx[k])
    print(f"fp32 path: eps rel-L2 {e:.3e}")
    worst = 0.0
    for k, (g, r) in checks.items():
        rr = rel(g, r)
        worst = max(worst, rr)
        print(f"  {k}: rel-L2 {rr:.3e}")
        assert rr < 1e-4, (k, rr)
    assert len(checks) == 18 and e < 1e-4
    print(f"worst gradient rel-L2 {worst:.3e}")


@pytest.mark.parametrize("cin,cout,h,rs", [(64, 64, 16, 0), (128, 256, 4, 2), (192, 64, 8, 0)])
def test_conv3x3_bwd_f32(dev, cin, cout, h, rs):
    """Conv input / weight / bias gradients of the fp32 GEMM forms (IM2COL x CONV_DGRAD,
    ROWM x IM2COL incl. the nearest-up gather) vs torch fp64 autograd."""
    from encdiff_amd import _lib as L, ops
    from encdiff_amd.ops import Geom
    g = torch.Generator().manual_seed(cin * 3 + cout)
    B = 2
    hs = h // 2 if rs == L.RESAMPLE_UP2 else h
    x = torch.randn(B, cin, hs, hs, generator=g, dtype=torch.float64, requires_grad=True)
    w = (torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * 0.05).requires_grad_(True)
    b = torch.randn(cout, generator=g, dtype=torch.float64, requires_grad=True)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if rs == L.RESAMPLE_UP2 else x
    y = F.conv2d(xin, w, b, padding=1)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(gy)
    go = Geom(B, h, h)
    rows = lambda t: t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).float().contiguous().to(dev)  # noqa: E731
    dy = rows(gy)
    wk = w.detach().permute(0, 2, 3, 1).reshape(cout, 9 * cin).float().contiguous().to(dev)
    dw = torch.zeros(cout, 9 * cin, device=dev)
    db = torch.zeros(cout, device=dev)
    ops.conv3x3_wgrad_f32(dy, rows(x.detach()), go, cin, dw, db=db, resample=rs)
    dxc = torch.empty(B * h * h, cin, device=dev)
    ops.conv3x3_dgrad_f32(dy, go, wk, dxc)
    if rs == L.RESAMPLE_UP2:
        dx = torch.empty(B * hs * hs, cin, device=dev)
        ops.ew_f32(L.EW_RESAMPLE_BWD, dxc, dx, resample=rs, g=Geom(B, hs, hs))
    else:
        dx = dxc
    r_w = rel(dw.cpu().view(cout, 3, 3, cin).permute(0, 3, 1, 2), w.grad)
    r_b = rel(db, b.grad)
    r_x = rel(dx.cpu().view(B, hs, hs, cin).permute(0, 3, 1, 2), x.grad)
    print(f"conv3x3 bwd fp32 {cin}->{cout} h{h} rs{rs}: dw {r_w:.2e} db {r_b:.2e} dx {r_x:.2e}")
    assert max(r_w, r_b, r_x) < 2e-6


def test_norm_attention_bwd_f32(dev):
    """GroupNorm(+FiLM+SiLU) / LayerNorm / attention backward (fp32 kernels) vs torch fp64 autograd."""
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    g = torch.Generator().manual_seed(9)
    d64 = dict(dtype=torch.float64)
    B, C, H = 2, 128, 8
    x = (torch.randn(B, C, H, H, generator=g, **d64) * 2 + 0.5).requires_grad_(True)
    gam = torch.randn(C, generator=g, **d64).requires_grad_(True)
    bet = torch.randn(C, generator=g, **d64).requires_grad_(True)
    film = (torch.randn(B, 2 * C, generator=g, **d64) * 0.3).requires_grad_(True)
    y = F.silu(F.group_norm(x, 32, gam, bet, 1e-5) * (1 + film[:, :C, None, None]) + film[:, C:, None, None])
    gy = torch.randn(y.shape, generator=g, **d64)
    y.backward(gy)
    rows = lambda t: t.detach().permute(0, 2, 3, 1).reshape(-1, t.shape[1]).float().contiguous().to(dev)  # noqa: E731
    xr = rows(x)
    yr = torch.empty_like(xr)
    st = torch.empty(B * 64, device=dev)
    ff = film.detach().float().to(dev)
    ops.groupnorm_f32(xr, Geom(B, H, H), gam.detach().float().to(dev), bet.detach().float().to(dev), yr, st, 1e-5,
                      True, film=ff, ld_film=2 * C)
    dx = torch.empty_like(xr)
    parts = torch.empty(B, 2 * C, device=dev)
    dfilm = torch.empty(B, 2 * C, device=dev)
    ops.groupnorm_bwd_f32(xr, Geom(B, H, H), gam.detach().float().to(dev), bet.detach().float().to(dev), st, True,
                          rows(gy), dx, parts[:, :C], parts[:, C:], 2 * C, film=ff, ld_film=2 * C, dfilm=dfilm,
                          ld_dfilm=2 * C)
    r = [rel(dx.cpu().view(B, H, H, C).permute(0, 3, 1, 2), x.grad), rel(parts[:, :C].sum(0), gam.grad),
         rel(parts[:, C:].sum(0), bet.grad), rel(dfilm, film.grad)]
    print("groupnorm bwd fp32 (dx, dgamma, dbeta, dfilm):", r)
    assert max(r) < 2e-6
    # LayerNorm over 300 rows
    t = (torch.randn(300, C, generator=g, **d64) * 2 - 0.5).requires_grad_(True)
    lt = F.layer_norm(t, (C,), gam, bet, 1e-5)
    gl = torch.randn(lt.shape, generator=g, **d64)
    gam.grad = bet.grad = None
    lt.backward(gl)
    tr = t.detach().float().contiguous().to(dev)
    lst = torch.empty(600, device=dev)
    ops.layernorm_f32(tr, gam.detach().float().to(dev), bet.detach().float().to(dev), torch.empty_like(tr), 1e-5,
                      stats=lst)
    dt = torch.empty_like(tr)
    lp = torch.empty(16, 2 * C, device=dev)
    ops.layernorm_bwd_f32(tr, gam.detach().float().to(dev), lst, gl.float().to(dev), dt, lp[:, :C], lp[:, C:], 16,
                          2 * C)
    r = [rel(dt, t.grad), rel(lp[:, :C].sum(0), gam.grad), rel(lp[:, C:].sum(0), bet.grad)]
    print("layernorm bwd fp32 (dx, dgamma, dbeta):", r)
    assert max(r) < 2e-6
    # attention (self at S = 64, cross to 20 keys), dh 16
    for sq, sk, dh in ((64, 64, 16), (64, 20, 32), (256, 256, 8)):
        h = 2
        q = torch.randn(B, sq, h * dh, generator=g, **d64).requires_grad_(True)
        k = torch.randn(B, sk, h * dh, generator=g, **d64).requires_grad_(True)
        v = torch.randn(B, sk, h * dh, generator=g, **d64).requires_grad_(True)
        split = lambda z: z.view(B, -1, h, dh).permute(0, 2, 1, 3)  # noqa: E731
        o = (torch.softmax(split(q) @ split(k).transpose(-1, -2) * dh ** -0.5, -1) @ split(v))
        o = o.permute(0, 2, 1, 3).reshape(B, sq, h * dh)
        go_ = torch.randn(o.shape, generator=g, **d64)
        o.backward(go_)
        f = lambda z: z.detach().reshape(-1, h * dh).float().contiguous().to(dev)  # noqa: E731
        qd, kd, vd = f(q), f(k), f(v)
        od = torch.empty_like(qd)
        lse = torch.empty(B * h * sq, device=dev)
        ops.attention_f32(qd, kd, vd, od, B, h, sq, sk, dh, lse=lse)
        dq, dk, dv = torch.empty_like(qd), torch.empty_like(kd), torch.empty_like(vd)
        ops.attention_bwd_f32(qd, kd, vd, od, lse, f(go_), dq, dk, dv, B, h, sq, sk, dh)
        r = [rel(dq, q.grad.reshape(-1, h * dh)), rel(dk, k.grad.reshape(-1, h * dh)), rel(dv, v.grad.reshape(-1, h * dh))]
        print(f"attention bwd fp32 sq{sq} sk{sk} dh{dh} (dq, dk, dv):", r)
        assert max(r) < 2e-6
