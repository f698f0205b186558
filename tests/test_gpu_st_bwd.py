"""The fused SpatialTransformer backward kernels alone (encdiff_st_tail_bwd / encdiff_st_head_bwd,
unet.UNetExecutor._st_bwd_fused) against a torch fp32 autograd restatement of the block
(attention.py:180-191 CrossAttention, :206-215 BasicTransformerBlock, :226-232 GEGLU, :250-261
SpatialTransformer) on the same bf16 operands: every gradient the kernels write (d_t3, d_f, d_t2,
d_q2, d_t1, d_o1; d_t0, d_gn), the concept tokens' dK / dV (one tile per image and several: the
ticket combine) and the LayerNorm affine gradients (the partial rows summed), at c = 64 / 128 and
the row tiles the UNet's levels use (an image over several tiles: per-tile slabs folded in tile order
by the head kernel's grid)."""
import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


def _bf(t):  # a stored bf16 tensor (autograd passes through the rounding)
    return t.bfloat16().float()


def _tail_case(c, hw, B, nctx, seed):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(seed)
    rows, h = B * hw, 8
    dh = c // h

    def r(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).bfloat16().float()
    W = {"out1": r(c, c, scale=c ** -0.5), "q2": r(c, c, scale=c ** -0.5), "out2": r(c, c, scale=c ** -0.5),
         "ff1": r(8 * c, c, scale=c ** -0.5), "ff2": r(c, 4 * c, scale=(4 * c) ** -0.5), "po": r(c, c, scale=c ** -0.5)}
    bvec = {k: 0.1 * torch.randn(n, device=dev, generator=g) for k, n in
            (("out1", c), ("out2", c), ("ff1", 8 * c), ("ff2", c), ("po", c))}
    g2 = (1 + 0.1 * torch.randn(c, device=dev, generator=g)).requires_grad_(True)
    be2 = (0.1 * torch.randn(c, device=dev, generator=g)).requires_grad_(True)
    g3 = (1 + 0.1 * torch.randn(c, device=dev, generator=g)).requires_grad_(True)
    be3 = (0.1 * torch.randn(c, device=dev, generator=g)).requires_grad_(True)
    o1 = r(rows, c).requires_grad_(True)
    t0, x = r(rows, c), r(rows, c)
    k2 = r(B * nctx, c).requires_grad_(True)
    v2 = r(B * nctx, c).requires_grad_(True)
    dy = r(rows, c, scale=0.1)
    # forward (fp32 arithmetic on the stored bf16 tensors, as the training forward saves them)
    t1 = _bf(o1 @ W["out1"].t() + bvec["out1"] + t0)
    m2, v2_ = t1.mean(1, keepdim=True), t1.var(1, unbiased=False, keepdim=True)
    n2 = _bf((t1 - m2) / torch.sqrt(v2_ + 1e-5) * g2 + be2)
    q2 = _bf(n2 @ W["q2"].t())
    qh = q2.view(B, hw, h, dh).permute(0, 2, 1, 3)
    kh = k2.view(B, nctx, h, dh).permute(0, 2, 1, 3)
    vh = v2.view(B, nctx, h, dh).permute(0, 2, 1, 3)
    s = qh @ kh.transpose(-1, -2) * dh ** -0.5
    lse = torch.logsumexp(s, -1)  # [B][h][hw]
    o2 = _bf((torch.softmax(s, -1) @ vh).permute(0, 2, 1, 3).reshape(rows, c))
    t2 = _bf(o2 @ W["out2"].t() + bvec["out2"] + t1)
    m3, v3 = t2.mean(1, keepdim=True), t2.var(1, unbiased=False, keepdim=True)
    n3 = _bf((t2 - m3) / torch.sqrt(v3 + 1e-5) * g3 + be3)
    f = _bf(n3 @ W["ff1"].t() + bvec["ff1"])
    a = _bf(f[:, :4 * c] * Fn.gelu(f[:, 4 * c:]))
    t3 = _bf(a @ W["ff2"].t() + bvec["ff2"] + t2)
    out = t3 @ W["po"].t() + bvec["po"] + x
    for t in (t1, q2, t2, f, t3):
        t.retain_grad()
    out.backward(dy)
    ref = dict(d_t3=t3.grad, d_f=f.grad, d_t2=t2.grad, d_q2=q2.grad, d_t1=t1.grad, d_o1=o1.grad, dk2=k2.grad,
               dv2=v2.grad, g3=g3.grad, be3=be3.grad, g2=g2.grad, be2=be2.grad)
    bfw = {k: v.bfloat16() for k, v in W.items()}
    save = dict(f=f.detach().bfloat16(), t2=t2.detach().bfloat16(), t1=t1.detach().bfloat16(),
                q2=q2.detach().bfloat16(), o2=o2.detach().bfloat16(),
                s3=torch.cat([m3, torch.rsqrt(v3 + 1e-5)], 1).detach().contiguous(),
                s2=torch.cat([m2, torch.rsqrt(v2_ + 1e-5)], 1).detach().contiguous(),
                lse2=lse.detach().reshape(B * h, hw).contiguous())
    return dict(c=c, hw=hw, B=B, nctx=nctx, rows=rows, W=bfw, g2=g2.detach(), g3=g3.detach(),
                k2=k2.detach().bfloat16(), v2=v2.detach().bfloat16(), dy=dy.bfloat16(), save=save, ref=ref)


def _run_tail(cs, parts):
    from encdiff_amd import ops
    dev, bf = "cuda", torch.bfloat16
    c, rows, B, nctx = cs["c"], cs["rows"], cs["B"], cs["nctx"]
    wt = {k: v.t().contiguous() for k, v in cs["W"].items() if k != "ff1"}
    wt["ff1"] = cs["W"]["ff1"].t().contiguous()  # [c][8c]
    out = {k: torch.empty(rows, c, device=dev, dtype=bf) for k in ("d_t3", "d_t2", "d_q2", "d_t1", "d_o1")}
    out["d_f"] = torch.empty(rows, 8 * c, device=dev, dtype=bf)
    pm = torch.full((parts, 4 * c), float("nan"), device=dev)
    ln3, ln2 = (pm[:, :c], pm[:, c:2 * c]), (pm[:, 2 * c:3 * c], pm[:, 3 * c:])
    dkv = torch.zeros(B * nctx, 2 * c, device=dev, dtype=bf)
    kv_part = torch.empty(rows // 32 * nctx, 2 * c, device=dev)
    ok = ops.st_tail_bwd(cs["dy"], cs["save"], wt, cs["g3"], cs["g2"], cs["k2"], cs["v2"], out, ln3, ln2,
                         dkv[:, :c], dkv[:, c:], rows, c, cs["hw"], 8, nctx, kv_part=kv_part)
    assert ok
    tile = ops.st_tail_bwd_tile(c, rows, cs["hw"])
    assert tile == (64 if c == 64 or (rows // 64 >= 256 and cs["hw"] % 64 == 0) else 32)
    tiles, tpi = rows // tile, cs["hw"] // tile
    if tpi > 1:  # the head kernel's grid folds the per-tile dK / dV slabs (its own outputs unused here)
        scratch = torch.empty(rows, c, device=dev, dtype=bf)
        pmh = torch.empty(rows // 32, 2 * c, device=dev)
        assert ops.st_head_bwd(torch.zeros(rows, 3 * c, device=dev, dtype=bf), scratch, scratch,
                               torch.ones(rows, 2, device=dev), cs["g3"], torch.zeros(c, 3 * c, device=dev, dtype=bf),
                               torch.zeros(c, c, device=dev, dtype=bf), scratch, scratch, (pmh[:, :c], pmh[:, c:]),
                               rows, c, kv=(kv_part, tpi, nctx, B, dkv[:, :c], dkv[:, c:]))
    torch.cuda.synchronize()
    got = dict(out, dk2=dkv[:, :c], dv2=dkv[:, c:], g3=ln3[0][:tiles].sum(0), be3=ln3[1][:tiles].sum(0),
               g2=ln2[0][:tiles].sum(0), be2=ln2[1][:tiles].sum(0))
    assert torch.isnan(pm[tiles:]).all() and not torch.isnan(pm[:tiles]).any()  # one partial row per tile
    return got


@pytest.mark.parametrize("c,hw,B,nctx", [(64, 256, 2, 20), (64, 256, 3, 40), (128, 64, 4, 20), (128, 64, 256, 20),
                                         (128, 1024, 2, 40)])
def test_st_tail_bwd_matches_autograd(c, hw, B, nctx):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cs = _tail_case(c, hw, B, nctx, seed=c * 7 + hw + B)
    got = _run_tail(cs, parts=cs["rows"] // 32 + 3)
    worst = 0.0
    for k, ref in cs["ref"].items():
        e = _rel(got[k], ref)
        worst = max(worst, e)
        print(f"c={c} hw={hw} B={B} nctx={nctx} {k}: rel-L2 {e:.2e}")
        # bf16 operands and stored gradients (as the per-layer launches store them) on the kernel side
        assert e < 2.5e-2, k
    # reproducible: a second launch gives the same bits (the dK / dV fold sums in tile order)
    again = _run_tail(cs, parts=cs["rows"] // 32 + 3)
    for k in got:
        assert torch.equal(got[k], again[k]), k


@pytest.mark.parametrize("c,hw,B", [(64, 256, 2), (64, 256, 128), (128, 64, 4)])
def test_st_head_bwd_matches_autograd(c, hw, B):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from encdiff_amd import ops
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(c + hw + B)
    rows = B * hw

    def r(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).bfloat16().float()
    w_in, w_qkv = r(c, c, scale=c ** -0.5), r(3 * c, c, scale=c ** -0.5)
    b_in = 0.1 * torch.randn(c, device=dev, generator=g)
    g1 = (1 + 0.1 * torch.randn(c, device=dev, generator=g)).requires_grad_(True)
    be1 = (0.1 * torch.randn(c, device=dev, generator=g)).requires_grad_(True)
    gn = r(rows, c).requires_grad_(True)
    d_qkv, d_t1 = r(rows, 3 * c, scale=0.1), r(rows, c, scale=0.1)
    t0 = _bf(gn @ w_in.t() + b_in)
    t0.retain_grad()
    m, v = t0.mean(1, keepdim=True), t0.var(1, unbiased=False, keepdim=True)
    n1 = _bf((t0 - m) / torch.sqrt(v + 1e-5) * g1 + be1)
    loss = ((n1 @ w_qkv.t()) * d_qkv).sum() + (t0 * d_t1).sum()
    loss.backward()
    parts = rows // 32 + 2
    pm = torch.full((parts, 2 * c), float("nan"), device=dev)
    d_t0 = torch.empty(rows, c, device=dev, dtype=bf)
    d_gn = torch.empty(rows, c, device=dev, dtype=bf)
    s1 = torch.cat([m, torch.rsqrt(v + 1e-5)], 1).detach().contiguous()
    ok = ops.st_head_bwd(d_qkv.bfloat16(), d_t1.bfloat16(), t0.detach().bfloat16(), s1, g1.detach(),
                         w_qkv.t().contiguous().bfloat16(), w_in.t().contiguous().bfloat16(), d_t0, d_gn,
                         (pm[:, :c], pm[:, c:]), rows, c)
    assert ok
    torch.cuda.synchronize()
    tiles = rows // (64 if c == 64 and rows // 64 >= 256 else 32)
    for name, got_, ref in (("d_t0", d_t0, t0.grad), ("d_gn", d_gn, gn.grad), ("g1", pm[:tiles, :c].sum(0), g1.grad),
                            ("be1", pm[:tiles, c:].sum(0), be1.grad)):
        e = _rel(got_, ref)
        print(f"c={c} hw={hw} B={B} {name}: rel-L2 {e:.2e}")
        assert e < 2e-2, name
    assert torch.isnan(pm[tiles:]).all() and not torch.isnan(pm[:tiles]).any()


@pytest.mark.parametrize("c,K", [(64, 32768), (128, 8192), (64, 256)])
def test_st_wgrad_matches_torch(c, K):
    """encdiff_st_wgrad (ops.StWgrad): the 8 weight gradients of a fused block in one grid + a chunk
    fold -- dW += dY^T X, db += sum dY -- vs torch fp32 on the same bf16 operands, accumulating onto
    prior values, and bitwise reproducible (chunk slabs summed in order).  K = 256: one chunk per
    block (accumulated in place, no fold)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from encdiff_amd import ops
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(c + K)
    shapes = [(c, c, True), (c, 4 * c, True), (8 * c, c, True), (c, c, True), (c, c, False), (c, c, True),
              (3 * c, c, False), (c, c, True)]  # (M = dY columns, N = X columns, bias)
    probs, refs = [], []
    for M, N, has_b in shapes:
        dy = (torch.randn(K, M, device=dev, generator=g) * 0.1).to(bf)
        x = torch.randn(K, N, device=dev, generator=g).to(bf)
        dw = torch.randn(M, N, device=dev, generator=g)
        db = torch.randn(M, device=dev, generator=g) if has_b else None
        refs.append((dw + dy.float().t() @ x.float(), db + dy.float().sum(0) if has_b else None))
        probs.append((dy, x, dw, db))
    init = [(dw.clone(), None if db is None else db.clone()) for _, _, dw, db in probs]
    wg = ops.StWgrad()
    wg.launch(probs)
    torch.cuda.synchronize()
    out1 = [(dw.clone(), None if db is None else db.clone()) for _, _, dw, db in probs]
    for (dw, db), (rw, rb) in zip(out1, refs):
        e = _rel(dw, rw)
        assert e < 1e-5, e
        if rb is not None:
            assert _rel(db, rb) < 1e-5
    # a second launch from the same initial values: the same bits
    for (_, _, dw, db), (w0, b0) in zip(probs, init):
        dw.copy_(w0)
        if db is not None:
            db.copy_(b0)
    wg.launch(probs)
    torch.cuda.synchronize()
    for (_, _, dw, db), (w1, b1) in zip(probs, out1):
        assert torch.equal(dw, w1) and (db is None or torch.equal(db, b1))


@pytest.mark.parametrize("c,K", [(64, 32768), (128, 8192)])
def test_st_wgrad_fold_rides_in_groupnorm_bwd(c, K):
    """StWgrad.launch(ride=True) launches only the weight-gradient grid; its chunk fold runs as extra
    workgroups of the next GroupNorm backward (groupnorm_bwd(fold=)).  Both results must be bitwise
    those of the separate launches (the fold sums the chunk slabs in the same order)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(5 * c + 1)
    shapes = [(c, c, True), (c, 4 * c, True), (8 * c, c, True), (3 * c, c, False)]
    probs = []
    for M, N, has_b in shapes:
        dy = (torch.randn(K, M, device=dev, generator=g) * 0.1).to(bf)
        x = torch.randn(K, N, device=dev, generator=g).to(bf)
        dw = torch.randn(M, N, device=dev, generator=g)
        db = torch.randn(M, device=dev, generator=g) if has_b else None
        probs.append((dy, x, dw, db))
    init = [(dw.clone(), None if db is None else db.clone()) for _, _, dw, db in probs]
    # a GroupNorm backward of the block's shape (B images of hw tokens, c channels)
    hw = 256 if c == 64 else 64
    B = K // hw
    gg = Geom(B, int(hw ** 0.5), int(hw ** 0.5))
    xg = (torch.randn(B * hw, c, device=dev, generator=g) + 0.3).to(bf)
    gam = 1 + 0.1 * torch.randn(c, device=dev, generator=g)
    bet = 0.1 * torch.randn(c, device=dev, generator=g)
    yg = torch.empty_like(xg)
    st = torch.empty(B, 32, 2, device=dev)
    ops.groupnorm_fwd(xg, gg, gam, bet, yg, st, 1e-6, False)
    dyg = (torch.randn(B * hw, c, device=dev, generator=g) * 0.1).to(bf)
    res = []
    for ride in (False, True):
        for (_, _, dw, db), (w0, b0) in zip(probs, init):
            dw.copy_(w0)
            if db is not None:
                db.copy_(b0)
        dx = torch.empty_like(xg)
        dgp = torch.empty(B, c, device=dev)
        dbp = torch.empty(B, c, device=dev)
        wg = ops.StWgrad()
        fold = wg.launch(probs, ride=ride)
        assert (fold is not None) == ride
        ops.groupnorm_bwd(xg, gg, gam, bet, st, 1e-6, False, dyg, dx, dgp, dbp, fold=fold)
        torch.cuda.synchronize()
        res.append(([dw.clone() for _, _, dw, _ in probs], [None if db is None else db.clone() for *_, db in probs],
                    dx, dgp, dbp))
    (w0, b0, dx0, g0, be0), (w1, b1, dx1, g1, be1) = res
    for a, b in zip(w0, w1):
        assert torch.equal(a, b)
    for a, b in zip(b0, b1):
        assert (a is None and b is None) or torch.equal(a, b)
    assert torch.equal(dx0, dx1) and torch.equal(g0, g1) and torch.equal(be0, be1)
    # and the gradients are right: dW = W0 + dY^T X
    for (dy, x, dw, db), (wi, bi), got in zip(probs, init, w1):
        assert _rel(got, wi + dy.float().t() @ x.float()) < 1e-5
