"""Run the fused ResNet-50 forward (bs=32) serially ITERS times, eagerly (one kernel per op), for
rocprofv3 counter collection over a whole forward:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 tools/probe/forward_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402


def main():
    batch = int(os.environ.get("BATCH", 32))
    iters = int(os.environ.get("ITERS", 3))
    dev = torch.device("cuda:0")
    model = ResNet50Fused(init_resnet50(0), dev, max_batch=batch, tuning=autotune.load_tuning("resnet50", batch, regime=os.environ.get("REGIME", "concurrent")))
    x = torch.randint(0, 256, (batch, 224, 224, 3), dtype=torch.uint8, device=dev)
    with torch.no_grad():
        conc = int(os.environ.get("CONC", "1"))
        if conc > 1:  # CONC graphs of the forward on CONC streams replayed together (the engine's regime)
            xs = [x.clone() for _ in range(conc)]
            ss = [torch.cuda.Stream(dev) for _ in range(conc)]
            gs = []
            for xi, si in zip(xs, ss):
                with torch.cuda.stream(si):
                    model.classify(xi, 5)
            torch.cuda.synchronize()
            for xi, si in zip(xs, ss):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(si), torch.cuda.graph(g, stream=si):
                    model.classify(xi, 5)
                gs.append(g)
            torch.cuda.synchronize()
            for _ in range(iters):
                for g, si in zip(gs, ss):
                    with torch.cuda.stream(si):
                        g.replay()
            torch.cuda.synchronize()
        elif os.environ.get("GRAPH") == "1":  # back-to-back replays of the captured forward: serial latency
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):  # eager warm-up on the capture stream (per-stream counters)
                model.classify(x, 5)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                model.classify(x, 5)
            torch.cuda.synchronize()
            for _ in range(iters):
                g.replay()
            torch.cuda.synchronize()
        else:
            for _ in range(iters):
                model.classify(x, 5)
                torch.cuda.synchronize()
    print("forwards", iters, flush=True)


if __name__ == "__main__":
    main()
