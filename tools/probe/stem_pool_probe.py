"""Fused stem (normalise + 7x7/2 conv + ReLU + 3x3/2 max pool, csrc/stem_pool.hip) vs the three-kernel
path at bs=32: graph-timed per call, alone and with 4 copies co-running."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.models.resnet import IMAGENET_MEAN, IMAGENET_STD  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402

dev = torch.device("cuda:0")
imgs = torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8, device=dev)
wp = ops.pack_conv_weight((torch.randn(64, 3, 7, 7, device=dev) * 0.05).to(torch.bfloat16))
bias = torch.randn(64, device=dev)
cfg, sk = autotune.load_tuning("resnet50", 32).get("stem", (0, 0))


def fused(o):
    return lambda: ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD, out=o)


def three(o, ws):
    xp = torch.empty(32, 230, 230, 4, device=dev, dtype=torch.bfloat16)
    y = torch.empty(32, 112, 112, 64, device=dev, dtype=torch.bfloat16)

    def run():
        ops.normalize_u8(imgs, IMAGENET_MEAN, IMAGENET_STD, pad=3, out=xp)
        ops.conv2d_nhwc(xp, wp, bias, kernel=7, stride=2, pad=0, act=ops.ACT_RELU, out=y, workspace=ws, cfg=cfg,
                        splitk=sk)
        ops.maxpool2d_nhwc(y, 3, 2, 1, out=o)
    return run


for conc in (1, 4):
    outs = [torch.empty(32, 56, 56, 64, device=dev, dtype=torch.bfloat16) for _ in range(conc)]
    wss = [torch.empty(1 << 20, device=dev, dtype=torch.float32) for _ in range(conc)]
    tf = autotune._time_multi([fused(o) for o in outs], 20)
    tt = autotune._time_multi([three(o, w_) for o, w_ in zip(outs, wss)], 20)
    print(json.dumps({"concurrency": conc, "fused_us": round(tf * 1e3, 2), "three_kernel_us": round(tt * 1e3, 2)}),
          flush=True)
