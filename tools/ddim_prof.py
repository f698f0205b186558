"""DDIM sampling alone (for rocprofv3 kernel statistics of the sampler step):
python tools/ddim_prof.py [--batch 8] [--steps 50] -- builds the Shapes3D LatentDiffusion,
runs DDIMSampler.sample twice (capture + timed) and prints steps/s."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--eta", type=float, default=0.0)
    a = ap.parse_args()
    import bench
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda().eval()
    print(f"DDIM B={a.batch} S={a.steps}: {bench.ddim_rate(ldm, a.batch, a.steps, a.eta):.1f} steps/s", flush=True)


if __name__ == "__main__":
    main()
