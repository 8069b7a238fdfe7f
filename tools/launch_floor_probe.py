"""Per-kernel cost floor inside a replayed hipGraph on this GPU: N dependent tiny launches (an
elementwise add on 1 KiB, and the native embedding kernel) captured once, replayed; µs per kernel.
Sets the budget for decode-step fusion work (how much a removed launch is worth).  JSON lines."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed_graph(fn, n_launch, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps / n_launch * 1e6


def main():
    from mlmicroservicetemplate_amd import ops

    dev = torch.device("cuda:0")
    x = torch.zeros(512, device=dev, dtype=torch.bfloat16)
    table = torch.randn(1024, 4096, device=dev).to(torch.bfloat16)
    ids = torch.zeros(1, device=dev, dtype=torch.int32)
    for n in (50, 200):
        def adds(n=n):
            for _ in range(n):
                x.add_(1)

        def embeds(n=n):
            for _ in range(n):
                ops.embedding(ids, table)

        print(json.dumps({"probe": "graph_launch_floor", "kernel": "torch add_ 512 el", "launches": n,
                          "us_per_kernel": round(timed_graph(adds, n), 2)}), flush=True)
        print(json.dumps({"probe": "graph_launch_floor", "kernel": "mls embedding 1x4096", "launches": n,
                          "us_per_kernel": round(timed_graph(embeds, n), 2)}), flush=True)


if __name__ == "__main__":
    main()
