"""Run selected ResNet-50 conv layers (bs=32) in isolation, for rocprofv3 counter collection.

    rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... --kernel-trace -- python3 tools/layer_probe.py stem layer1.0.conv3
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.models.resnet import conv_shapes  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402


def main():
    names = sys.argv[1:] or ["stem", "layer1.0.conv1", "layer1.0.conv3", "layer3.1.conv2"]
    batch = int(os.environ.get("BATCH", 32))
    iters = int(os.environ.get("ITERS", 10))
    tuning = autotune.load_tuning("resnet50", batch)
    dev = torch.device("cuda:0")
    ws = torch.empty(64 << 20, device=dev, dtype=torch.float32)
    shapes = {s.name: (s, hin, ho) for s, hin, ho in conv_shapes()}
    for name in names:
        s, hin, ho = shapes[name]
        cin = 4 if s.name == "stem" else s.cin
        hp = hin + 6 if s.name == "stem" else hin
        x = torch.randn(batch, hp, hp, cin, device=dev).to(torch.bfloat16)
        w = ops.pack_conv_weight((torch.randn(s.cout, s.cin, s.k, s.k, device=dev) * 0.05).to(torch.bfloat16))
        b = torch.randn(s.cout, device=dev)
        res = torch.randn(batch, ho, ho, s.cout, device=dev).to(torch.bfloat16) if name.endswith("conv3") else None
        cfg, sk = tuning.get(name, (0, 0))
        cfg = int(os.environ.get("CFG", cfg))
        sk = int(os.environ.get("SPLITK", sk))
        for _ in range(iters):
            ops.conv2d_nhwc(x, w, b, kernel=s.k, stride=s.stride, pad=0 if s.name == "stem" else s.pad, residual=res, act=1, workspace=ws,
                            cfg=cfg, splitk=sk)
        torch.cuda.synchronize()
        print(name, "cfg", cfg, "splitk", sk, flush=True)


if __name__ == "__main__":
    main()
