"""Which torch (non-encdiff) GPU kernels run inside one training step, and which Python line
launched each (torch.profiler, eager step).

    python tools/torch_kernels.py [--batch 128]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

OURS = ("gemm", "gn_", "ln_", "attn_", "st_", "ew_kernel", "bn_", "warp_", "small_conv", "temb", "qsample", "l1_",
        "adamw", "pack_", "reduce_partials", "gather_u8", "counter_inc", "nchw_to_rows", "grad_fold", "ddim")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    import bench
    from encdiff_amd.trainer import HipTrainer
    from torch.profiler import ProfilerActivity, profile
    ldm, _ = bench.build_ldm("shapes3d")
    tr = HipTrainer(ldm, a.batch, graph=False, pool_size=4 * a.batch)
    tr.init_scale_factor()
    for _ in range(2):
        tr.step_eager()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.step_eager()
        torch.cuda.synchronize()
    evs = prof.events()
    by_id = {e.id: e for e in evs}
    n = 0
    for e in evs:
        if e.device_type != torch.autograd.DeviceType.CUDA:
            continue
        if any(k in e.name for k in OURS):
            continue
        n += 1
        p = e.cpu_parent if hasattr(e, "cpu_parent") else None
        chain = []
        while p is not None and len(chain) < 3:
            chain.append(p.name)
            p = p.cpu_parent
        st = ""
        q = e.cpu_parent
        while q is not None:
            if q.stack:
                st = " <- ".join(s for s in q.stack if "encdiff_amd" in s or "trainer" in s)[:400]
                break
            q = q.cpu_parent
        print(f"{e.name[:70]:70s} | {' / '.join(chain)[:80]} | {st}")
    print("torch kernels per step:", n)


if __name__ == "__main__":
    main()
