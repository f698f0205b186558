"""Time the as-is PyTorch stages of the step (graph-captured) under execution modes:
frozen VQ encoder fp32 / bf16-autocast / bf16-autocast channels_last, and Encoder4
fwd+bwd fp32 / bf16-autocast.  Informs the configuration of HipTrainer."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_time(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    torch.backends.cudnn.benchmark = True
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    B = 128
    img = torch.rand(B, 3, 64, 64, device="cuda") * 2 - 1
    fs = ldm.first_stage_model
    with torch.no_grad():
        ref = fs.encode(img)
    print(f"vq fp32 NCHW          {graph_time(lambda: fs.encode(img)):7.3f} ms")

    def vq_bf16():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return fs.encode(img)
    with torch.no_grad():
        z = vq_bf16().float()
        print(f"vq bf16 rel-L2 {((z - ref).norm() / ref.norm()).item():.3e}")
        print(f"vq bf16 NCHW          {graph_time(vq_bf16):7.3f} ms")
        fs_cl = fs.to(memory_format=torch.channels_last)
        img_cl = img.contiguous(memory_format=torch.channels_last)

        def vq_bf16_cl():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return fs_cl.encode(img_cl)
        print(f"vq bf16 NHWC          {graph_time(vq_bf16_cl):7.3f} ms")
        fs.to(memory_format=torch.contiguous_format)
    enc = ldm.cond_stage_model
    enc.train()
    gout = torch.randn(B, 320, device="cuda")

    def e4():
        c = enc(img)
        c.backward(gout)
    print(f"encoder4 fwd+bwd fp32 {graph_time(e4):7.3f} ms")

    def e4f():
        with torch.no_grad():
            enc(img)
    print(f"encoder4 fwd fp32     {graph_time(e4f):7.3f} ms")

    def e4_bf16():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            c = enc(img)
        c.float().backward(gout)
    print(f"encoder4 fwd+bwd bf16 {graph_time(e4_bf16):7.3f} ms")

    def warp_only():
        u = torch.randn(B, 20, device="cuda", requires_grad=True)
        enc.warp(u).backward(gout)
    print(f"encoder4 warp fwd+bwd {graph_time(warp_only):7.3f} ms")


if __name__ == "__main__":
    main()
