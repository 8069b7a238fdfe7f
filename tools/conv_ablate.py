"""Ablation timing of the conv kernel on ResNet-50 layers (diagnostics; guide §7 'The diagnostic
loop'): full kernel vs no-MFMA (1) vs no-store (2) vs no-operand-DMA (4) vs combinations."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.models.resnet import conv_shapes  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402


def main():
    names = sys.argv[1:] or ["stem", "layer1.0.conv1", "layer1.0.conv2", "layer1.0.conv3", "layer2.1.conv1",
                             "layer2.0.conv3", "layer3.1.conv2", "layer3.1.conv3", "layer4.1.conv2"]
    batch = 32
    tuning = autotune.load_tuning("resnet50", batch)
    dev = torch.device("cuda:0")
    ws = torch.empty(64 << 20, device=dev, dtype=torch.float32)
    shapes = {s.name: (s, hin, ho) for s, hin, ho in conv_shapes()}
    L = ops.lib()
    for name in names:
        s, hin, ho = shapes[name]
        cin = 4 if s.name == "stem" else s.cin
        hp = hin + 6 if s.name == "stem" else hin
        x = torch.randn(batch, hp, hp, cin, device=dev).to(torch.bfloat16)
        w = ops.pack_conv_weight((torch.randn(s.cout, s.cin, s.k, s.k, device=dev) * 0.05).to(torch.bfloat16))
        b = torch.randn(s.cout, device=dev)
        res = torch.randn(batch, ho, ho, s.cout, device=dev).to(torch.bfloat16) if name.endswith("conv3") else None
        out = torch.empty(batch, ho, ho, s.cout, device=dev, dtype=torch.bfloat16)
        cfg, sk = tuning.get(name, (0, 0))
        row = {"layer": name, "cfg": cfg, "splitk": sk}
        for flags in (0, 1, 2, 4, 3, 5, 6, 7):
            L.mls_set_debug_flags(flags)
            t = autotune._time(lambda: ops.conv2d_nhwc(x, w, b, kernel=s.k, stride=s.stride,
                                                       pad=0 if s.name == "stem" else s.pad, residual=res, act=1,
                                                       out=out, workspace=ws, cfg=cfg, splitk=sk), iters=30)
            row[f"f{flags}"] = round(t * 1e3, 2)
        L.mls_set_debug_flags(0)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
