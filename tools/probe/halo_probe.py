"""Halo-tiled direct 3x3 (csrc/conv3x3_halo.hip) vs the tuned implicit-GEMM conv on the four
ResNet-50 bottleneck conv2 shapes at bs=32, graph-timed per call alone and with 4 copies co-running."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402

dev = torch.device("cuda:0")
tuning = autotune.load_tuning("resnet50", 32)
B = 32
for layer, (H, C) in {"layer1.1.conv2": (56, 64), "layer2.1.conv2": (28, 128), "layer3.1.conv2": (14, 256),
                      "layer4.1.conv2": (7, 512)}.items():
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    w = ops.pack_conv_weight((torch.randn(C, C, 3, 3, device=dev) * 0.02).to(torch.bfloat16))
    b = torch.randn(C, device=dev) * 0.1
    cfg, sk = tuning.get(layer, (0, 0))
    for conc in (1, 4):
        outs = [torch.empty(B, H, H, C, device=dev, dtype=torch.bfloat16) for _ in range(conc)]
        wss = [torch.empty(8 << 20, device=dev, dtype=torch.float32) for _ in range(conc)]
        th = autotune._time_multi([lambda o=o: ops.conv3x3_halo(x, w, b, act=ops.ACT_RELU, out=o) for o in outs], 20)
        tg = autotune._time_multi([lambda o=o, ws=ws: ops.conv2d_nhwc(x, w, b, kernel=3, stride=1, pad=1,
                                                                      act=ops.ACT_RELU, out=o, workspace=ws, cfg=cfg,
                                                                      splitk=sk) for o, ws in zip(outs, wss)], 20)
        fl = 2 * B * H * H * C * C * 9
        print(json.dumps({"layer": layer, "concurrency": conc, "geometry": ops.conv3x3_halo_geometry(B, H, H),
                          "halo_us": round(th * 1e3, 2), "gemm_us": round(tg * 1e3, 2), "gemm_cfg": [cfg, sk],
                          "halo_tflops": round(fl / th / 1e9, 1), "gemm_tflops": round(fl / tg / 1e9, 1)}),
              flush=True)
