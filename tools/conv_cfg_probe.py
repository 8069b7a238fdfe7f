"""Graph-timed µs of chosen ResNet-50 conv layers (bs=32) under every kernel config, isolated and
with 2 batches co-running -- which tile / pipeline shapes win where.  JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import conv_shapes
    from mlmicroservicetemplate_amd.ops.autotune import _time_multi

    layers = sys.argv[1:] or ["layer1.0.conv1", "layer1.0.conv2", "layer1.0.conv3", "layer1.0.down",
                              "layer2.1.conv2", "layer3.1.conv2", "layer3.1.conv3"]
    dev = torch.device("cuda:0")
    shapes = {s.name: (s, hin, ho) for s, hin, ho in conv_shapes()}
    for name in layers:
        s, hin, ho = shapes[name]
        x = torch.randn(32, hin, hin, s.cin, device=dev).to(torch.bfloat16)
        w = ops.pack_conv_weight((torch.randn(s.cout, s.cin, s.k, s.k, device=dev) * 0.05).to(torch.bfloat16))
        b = torch.randn(s.cout, device=dev)
        res = torch.randn(32, ho, ho, s.cout, device=dev).to(torch.bfloat16) if name.endswith("conv3") else None
        outs = [torch.empty(32, ho, ho, s.cout, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        wss = [torch.empty(64 << 20, device=dev) for _ in range(2)]
        for cfg in list(range(1, 19)) + [20, 21, 22]:
            row = {"layer": name, "cfg": cfg}
            for conc in (1, 2):
                fns = [lambda o=o, wsc=wsc: ops.conv2d_nhwc(x, w, b, kernel=s.k, stride=s.stride, pad=s.pad,
                                                            residual=res, act=1, out=o, workspace=wsc, cfg=cfg,
                                                            splitk=1) for o, wsc in zip(outs[:conc], wss[:conc])]
                try:
                    row[f"us_c{conc}"] = round(_time_multi(fns, 20) * 1e3, 2)
                except Exception as e:
                    row[f"us_c{conc}"] = None
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
