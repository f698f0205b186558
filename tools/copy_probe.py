"""Which host calls issue device copies in one B=8 UNet forward (torch profiler, Python stacks).

    python tools/copy_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda().eval()
    x = torch.randn(8, 3, 16, 16, device="cuda")
    t = torch.full((8,), 500, device="cuda", dtype=torch.long)
    c = torch.randn(8, 20, 16, device="cuda")
    with torch.no_grad():
        for _ in range(2):
            ldm.apply_model(x, t, c)
        torch.cuda.synchronize()
        from torch.profiler import profile, ProfilerActivity
        with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
            ldm.apply_model(x, t, c)
            torch.cuda.synchronize()
    n = 0
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::to", "aten::_to_copy", "aten::cat",
                       "aten::index_select", "aten::zeros", "aten::fill_", "aten::zero_"):
            n += 1
            stack = [s for s in ev.stack if "encdiff_amd" in s or "tools" in s][:4]
            print(ev.name, ev.input_shapes[:2], " <- ", " | ".join(stack))
    print("events:", n)


if __name__ == "__main__":
    main()
