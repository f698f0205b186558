"""Does a captured HIP graph run independent branches concurrently?

    python tools/graph_concurrency.py

Two chains of N small GEMMs (32 workgroups each, latency-bound): captured on one stream,
then forked onto two streams inside the capture.  Prints the replay time of each form and
of the same work launched eagerly on two streams.
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from encdiff_amd import ops
    dev = "cuda"
    bf = torch.bfloat16
    N = 20
    M, K, Nn = 512, 256, 256
    xs = [torch.randn(M, K, device=dev).to(bf) for _ in range(2)]
    w = (torch.randn(Nn, K, device=dev) * 0.05).to(bf)
    ys = [torch.empty(M, Nn, device=dev, dtype=bf) for _ in range(2)]
    side = torch.cuda.Stream()

    def chain(i):
        for _ in range(N):
            ops.linear_fwd(xs[i], w, ys[i])

    def one_stream():
        chain(0)
        chain(1)

    def two_streams():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            chain(1)
        chain(0)
        main.wait_stream(side)

    def two_streams_split(k):
        # k forks: chain 1 is cut into k pieces, each forked after a piece of chain 0
        main = torch.cuda.current_stream()
        for j in range(k):
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for _ in range(N // k):
                    ops.linear_fwd(xs[1], w, ys[1])
            for _ in range(N // k):
                ops.linear_fwd(xs[0], w, ys[0])
        main.wait_stream(side)

    def timed_graph(fn, reps=20):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
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

    def timed_eager(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    print(f"graph one stream      {timed_graph(one_stream):8.1f} us  ({2 * N} GEMMs)")
    print(f"graph two streams     {timed_graph(two_streams):8.1f} us")
    for k in (2, 5, 10, 20):
        print(f"graph two streams x{k:<2d} {timed_graph(lambda: two_streams_split(k)):8.1f} us")
    print(f"eager one stream      {timed_eager(one_stream):8.1f} us")
    print(f"eager two streams     {timed_eager(two_streams):8.1f} us")


if __name__ == "__main__":
    main()
