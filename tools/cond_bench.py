"""Time the as-is stages of the step in isolation (each replayed from a HIP graph):
Encoder4 forward+backward in fp32 (reference precision), bf16 autocast and channels-last
variants, and the frozen VQ encoder.

    python tools/cond_bench.py [--batch 128]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    B = a.batch
    img = torch.rand(B, 3, 64, 64, device="cuda") * 2 - 1
    enc = ldm.cond_stage_model
    enc.train()
    d = torch.randn(B, 320, device="cuda")

    def e4(dtype=None, cl=False):
        x = img.contiguous(memory_format=torch.channels_last) if cl else img
        trunk = enc.encoder[:-2]  # up to View((-1, 2048)) + Linear
        if dtype is None:
            c = trunk(x)
        else:
            with torch.autocast("cuda", dtype=dtype):
                c = trunk(x)
        c.float().sum().backward()

    print(f"Encoder4 conv trunk fwd+bwd fp32          {timed(lambda: e4()):8.1f} us")
    enc.to(memory_format=torch.channels_last)
    print(f"Encoder4 conv trunk fwd+bwd fp32 NHWC     {timed(lambda: e4(cl=True)):8.1f} us")
    print(f"Encoder4 conv trunk fwd+bwd bf16 NHWC     {timed(lambda: e4(torch.bfloat16, True)):8.1f} us")
    enc.to(memory_format=torch.contiguous_format)
    print(f"Encoder4 conv trunk fwd+bwd bf16 NCHW     {timed(lambda: e4(torch.bfloat16)):8.1f} us")

    def full():
        c = ldm.get_learned_conditioning(img)
        c.backward(d)
    print(f"Encoder4 full (trunk + warp) fwd+bwd     {timed(full):8.1f} us")
    with torch.no_grad():
        print(f"VQ encode (HIP)                           "
              f"{timed(lambda: ldm.get_first_stage_encoding(ldm.encode_first_stage(img))):8.1f} us")


if __name__ == "__main__":
    main()
