"""Time encdiff_encoder_head_bwd (Encoder4's final Linear backward) alone at the training batch,
graph-replayed; with ENCDIFF_LIB pointing at a -DHEADBWD_SKIP=<mask> build, per part.

    python tools/head_bwd_bench.py [--batch 128] [--d 128] [--units 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--units", type=int, default=20)
    a = ap.parse_args()
    from encdiff_amd import _lib as L, ops
    from gn_bench import timed
    B, d, U = a.batch, a.d, a.units
    r1 = torch.randn(B * 16, d, device="cuda")
    W = torch.randn(U, d * 16, device="cuda")
    du = torch.randn(B, U, device="cuda")
    dh = torch.empty(B * 16, d, device="cuda", dtype=torch.bfloat16)
    dW = torch.zeros(U, d * 16, device="cuda")
    db = torch.zeros(U, device="cuda")

    def run():
        L.check(L.lib.encdiff_encoder_head_bwd(r1.data_ptr(), r1.stride(0), B, d, W.data_ptr(), U, du.data_ptr(),
                                               du.stride(0), dh.data_ptr(), dh.stride(0), dW.data_ptr(),
                                               db.data_ptr(), ops._s()), "head_bwd")
    print(f"head_bwd B={B} d={d} units={U}: {timed(run):.2f} us", flush=True)


if __name__ == "__main__":
    main()
