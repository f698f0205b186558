"""encdiff_st_head_fwd alone (attention.py:250-254 + :211 norm1, the q/k/v projections): GroupNorm32
from x (the kernel's own statistics, inference), proj_in + bias, LayerNorm, q/k/v -- against a torch
fp32 restatement on the same bf16 operands, at every SpatialTransformer width of the UNet and the
sampling tiles (c = 256: the 8-wave form that streams its weights)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x, gn_w, gn_b, w_in, b_in, g1, be1, w_qkv, B, tokens, c):
    xf = x.float().view(B, tokens, 32, c // 32)
    m = xf.mean(dim=(1, 3), keepdim=True)
    v = xf.var(dim=(1, 3), unbiased=False, keepdim=True)
    gn = ((xf - m) / torch.sqrt(v + 1e-6)).view(B * tokens, c) * gn_w + gn_b
    gn = gn.bfloat16().float()
    t0 = (gn @ w_in.float().t() + b_in).bfloat16().float()  # stored bf16, LN1 reads the stored values
    n1 = torch.nn.functional.layer_norm(t0, (c,), g1, be1, 1e-5).bfloat16().float()
    return t0, n1 @ w_qkv.float().t()


@pytest.mark.parametrize("c,hw", [(64, 256), (128, 64), (256, 16), (256, 4)])
@pytest.mark.parametrize("B", [2, 8])
def test_st_head_matches_restatement(c, hw, B):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from encdiff_amd import ops
    g = torch.Generator(device="cuda").manual_seed(c + hw + B)
    dev, bf = "cuda", torch.bfloat16

    def r(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(bf)
    rows = B * hw
    x = r(rows, c)
    w_in, w_qkv = r(c, c, scale=c ** -0.5), r(3 * c, c, scale=c ** -0.5)
    gn_w = 1 + 0.1 * torch.randn(c, device=dev, generator=g)
    gn_b = 0.1 * torch.randn(c, device=dev, generator=g)
    b_in = 0.1 * torch.randn(c, device=dev, generator=g)
    g1 = 1 + 0.1 * torch.randn(c, device=dev, generator=g)
    be1 = 0.1 * torch.randn(c, device=dev, generator=g)
    t0 = torch.empty(rows, c, device=dev, dtype=bf)
    qkv = torch.empty(rows, 3 * c, device=dev, dtype=bf)
    gn = torch.empty(rows, c, device=dev, dtype=bf)
    ok = ops.st_head_fwd(x, gn, w_in, b_in, g1, be1, w_qkv, t0, qkv, rows, c, hw, 1e-6, 1e-5,
                         gn_gamma=gn_w, gn_beta=gn_b, self_stats=True)
    if rows % 16:  # a 16-row tile would span a partial image group: declined, the caller runs the launches
        assert not ok
        return
    assert ok, "the fused head declined a sampling-tile shape"
    torch.cuda.synchronize()
    t0_ref, qkv_ref = _ref(x, gn_w, gn_b, w_in, b_in, g1, be1, w_qkv, B, hw, c)
    for name, got, ref in (("t0", t0.float(), t0_ref), ("qkv", qkv.float(), qkv_ref)):
        rel = ((got - ref).norm() / ref.norm()).item()
        mab = (got - ref).abs().max().item()
        print(f"c={c} hw={hw} B={B} {name}: rel-L2 {rel:.2e} max-abs {mab:.2e}")
        # bf16 operands / outputs on both sides; differences are roundings at different points
        assert rel < 1e-2 and mab < 0.1 * ref.abs().max().item()
