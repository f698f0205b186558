"""Determinism probe: the same eager fwd+bwd (fed inputs) repeated in one process must give
bitwise identical arena gradients; prints the parameters that differ."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    torch.manual_seed(1234)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    ldm.use_scheduler = False
    tr = HipTrainer(ldm, B, base_lr=1e-4 / B, pool_size=4 * B)
    f = tr.enable_feed()
    g = torch.Generator().manual_seed(5)
    f["img"].copy_(torch.rand(B, 3, 64, 64, generator=g) * 2 - 1)
    f["t"].copy_(torch.randint(0, 1000, (B,), generator=g))
    f["noise"].copy_(torch.randn(B, 3, 16, 16, generator=g))
    tr.init_scale_factor()
    a = tr.arena
    ref = None
    for rep in range(6):
        tr._fwd_bwd()
        torch.cuda.synchronize()
        gr = a.grad.clone()
        if ref is None:
            ref = gr
            continue
        bad = [(n, float((a.view_in(gr, n) - a.view_in(ref, n)).abs().max())) for n in a.names
               if not torch.equal(a.view_in(gr, n), a.view_in(ref, n))]
        print(f"rep {rep}: {len(bad)} parameters differ {bad[:8]}", flush=True)


if __name__ == "__main__":
    main()
