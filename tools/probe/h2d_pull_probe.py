"""Zero-copy H2D (ops.h2d_pull, csrc/engine_launch.hip) vs hipMemcpyAsync (SDMA) for one ResNet
batch (32 x 224 x 224 x 3 uint8 = 4.8 MB): device time per copy, alone and beside a co-running
ResNet-50 forward on another stream."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlmicroservicetemplate_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
src = torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8).pin_memory()
dst = torch.empty(src.shape, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(dev)


def timed(fn, n=50):
    with torch.cuda.stream(s):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            fn()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = {"sdma_us": round(timed(lambda: dst.copy_(src, non_blocking=True)), 1)}
for blocks in (2, 4, 8, 16, 32):
    res[f"pull{blocks}_us"] = round(timed(lambda b=blocks: ops.h2d_pull(src, dst, b)), 1)
ok = torch.equal(dst.cpu(), src)
print(json.dumps({"bytes": src.numel(), "equal": ok, **res}), flush=True)
