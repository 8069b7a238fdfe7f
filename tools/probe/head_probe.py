"""Fused head (csrc/head.hip fc_head_kernel) alone, graph-timed per call: k = 5 (FC + softmax +
top-k) vs k = 0 (FC only, no finisher), at B = 32 / 8 / 4 -- where the kernel's time goes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402

dev = torch.device("cuda:0")
w = (torch.randn(1000, 2048) * 0.03).to(torch.bfloat16).to(dev)
b = (torch.randn(1000) * 0.1).to(dev)
for B in (32, 8, 4):
    pooled = (torch.rand(B, 2048) * 2).to(dev)
    logits = torch.empty(B, 1000, device=dev)
    vals = torch.empty(B, 5, device=dev)
    idx = torch.empty(B, 5, device=dev, dtype=torch.int32)
    res = {"B": B}
    for k in (5, 0):
        fn = lambda k=k: ops.fc_head(pooled, w, b, k, logits=logits, vals=vals, idx=idx)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        res[f"k{k}_us"] = round(autotune._time_multi([fn], 50) * 1e3, 2)
    print(json.dumps(res), flush=True)
