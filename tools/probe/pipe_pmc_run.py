"""Runs the 3x3 conv candidates a few times each (for rocprofv3 --pmc): layer1 / layer3 shapes,
the round-1 halo kernel vs the pipelined kernel."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mlmicroservicetemplate_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
B = 32
for H, C, cands in ((56, 64, [(100, 1), (113, 17)]), (14, 256, [(100, 1), (111, 1), (113, 1)])):
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    w = ops.pack_conv_weight((torch.randn(C, C, 3, 3, device=dev) * 0.02).to(torch.bfloat16))
    b = torch.randn(C, device=dev) * 0.1
    ws = torch.empty(4 * B * H * H * C, device=dev)
    for cfg, sk in cands:
        for _ in range(int(os.environ.get("ITERS", 5))):
            ops.conv2d_nhwc(x, w, b, kernel=3, stride=1, pad=1, act=ops.ACT_RELU, workspace=ws, cfg=cfg, splitk=sk)
        torch.cuda.synchronize()
