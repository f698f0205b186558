"""Which parameter gradients differ between the deferred split-K finalize fused into the norms
(unet.GN_FIN = True) and separate finalize launches (False) at B = 64: per parameter max-abs
difference, in backward order (output side first).  Diagnostic for test_unet_gn_fin_bitwise.

    python tools/gnfin_diag.py
"""
from __future__ import annotations

import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from encdiff_amd import unet as U
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    from oracle import encdiff_oracle as O
    m = UNetModel(**O.SHAPES3D_UNET)
    m.load_state_dict(O.recipe_params(O.param_shapes(O.build_plan())), strict=True)
    m = m.cuda()
    torch.manual_seed(29)
    B = 64
    x = torch.randn(B, 3, 16, 16, device="cuda")
    t = torch.randint(0, 1000, (B,), device="cuda")
    c = torch.randn(B, 320, device="cuda")
    g = torch.randn(B, 3, 16, 16, device="cuda")
    U.AGN = False
    out = {}
    for on in (True, False, True):
        U.GN_FIN = on
        m.executor()
        m._arena.zero_grad()
        cc = c.clone().requires_grad_(True)
        eps = m(x, t, context=[cc])
        eps.backward(g)
        torch.cuda.synchronize()
        out.setdefault(on, []).append((eps.detach().clone(), {k: p.grad.clone() for k, p in m.named_parameters()},
                                       cc.grad.clone()))
    a, b, a2 = out[True][0], out[False][0], out[True][1]
    print("eps equal:", torch.equal(a[0], b[0]), " run-to-run (fused twice) grads equal:",
          all(torch.equal(a[1][k], a2[1][k]) for k in a[1]))
    print("dctx max-abs diff:", (a[2] - b[2]).abs().max().item())
    names = list(a[1].keys())
    for k in reversed(names):
        d = (a[1][k] - b[1][k]).abs().max().item()
        if d > 0:
            print(f"{k:70s} {d:.3e}  (|g| max {b[1][k].abs().max().item():.3e})")


if __name__ == "__main__":
    main()
