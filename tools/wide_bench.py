"""UNet forward+backward throughput of the wider builder-defined UNet of BASELINE.json
configs[4] (32x32 latent, model_channels 128, 40 concept tokens; tests/test_gpu_unet_wide.py)
on one MI355X.  Only the denoiser: the 128x128 VQ encoder / Encoder4 of that config are
not part of the measurement.  Prints one JSON line (imgs/s, ms per fwd+bwd, TFLOP/s from
the torch FlopCounter count of the oracle forward x 3).

usage: python tools/wide_bench.py [--batch 64] [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import encdiff_amd  # noqa: F401
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    from oracle import encdiff_oracle as O
    from test_gpu_unet_wide import WIDE_UNET
    from torch.utils.flop_counter import FlopCounterMode

    plan = O.build_plan(WIDE_UNET)
    P = O.recipe_params(O.param_shapes(plan))
    with FlopCounterMode(display=False) as fc, torch.no_grad():
        O.unet_forward(P, plan, torch.randn(1, 3, 32, 32), torch.tensor([5]), [torch.randn(1, 640)])
    f_fwd = fc.get_total_flops()
    m = UNetModel(**WIDE_UNET)
    m.load_state_dict(P, strict=True)
    m = m.cuda()
    B = args.batch
    x = torch.randn(B, 3, 32, 32, device="cuda")
    t = torch.randint(0, 1000, (B,), device="cuda")
    c = torch.randn(B, 640, device="cuda", requires_grad=True)
    g = torch.randn(B, 3, 32, 32, device="cuda")
    m.executor()

    def step():
        m._arena.zero_grad()
        m(x, t, context=[c]).backward(g)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    tf = 3 * f_fwd * B / dt / 1e12
    print(json.dumps({"workload": "configs[4] wide UNet fwd+bwd (32x32 latent, mc 128, 40 tokens), eager",
                      "batch": B, "ms_per_step": dt * 1e3, "imgs_per_s": B / dt,
                      "gflop_fwd_per_img": f_fwd / 1e9, "tflops": tf, "frac_bf16_peak": tf / 2500.0}))


if __name__ == "__main__":
    main()
