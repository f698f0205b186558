"""Debug: out.2.bias gradient at B=512 (eager step vs graph replay vs host sum of the seed)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.step_check import GraphStepCheck

for B in (int(a) for a in sys.argv[1:] or ["512"]):
    chk = GraphStepCheck(B=B, seed=512, warmup=1)
    tr, a = chk.tr, chk.tr.arena
    img, t, noise = chk.inputs()
    chk._put(img, t, noise)
    for mode in ("graph", "eager"):
        if mode == "graph":
            tr.step()
        else:
            tr.step_eager()
        torch.cuda.synchronize()
        eps = tr.unet._ex.eps.detach().cpu()
        seed = torch.sign(eps - noise) / eps.numel()
        want = seed.double().sum((0, 2, 3))
        got = a.view_in(a.grad, "out.2.bias").detach().cpu()
        print(B, mode, "out.2.bias grad", got.tolist(), "host sum of seed", want.tolist(), flush=True)
    # torch reduction inside a captured graph at this size
    d = torch.randn(B, 3, 16, 16, device="cuda")
    o = torch.zeros(3, device="cuda")
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        o.add_(d.sum((0, 2, 3)))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            o.zero_(); o.add_(d.sum((0, 2, 3)))
    torch.cuda.current_stream().wait_stream(s)
    g.replay(); torch.cuda.synchronize()
    print(B, "torch sum in graph", o.tolist(), "eager", d.sum((0, 2, 3)).tolist(), flush=True)
    del chk
