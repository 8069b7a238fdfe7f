"""1x1 stride-1 ResNet-50 convs (bs=32) as plain GEMMs: the shipped native (cfg, split-K) vs
hipBLASLt (torch._addmm_activation: bias + ReLU epilogue; conv3: addmm with the residual as C,
then the bias+ReLU as a separate pass), per-call cost with `--concurrency` copies co-running."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd.models.resnet import conv_shapes  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune, conv2d_nhwc, pack_conv_weight  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=4)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tuning = autotune.load_tuning("resnet50", a.batch)
    ws = [torch.empty(64 << 20, device=dev, dtype=torch.float32) for _ in range(a.concurrency)]
    seen = set()
    for s, hin, ho in conv_shapes():
        if s.k != 1 or s.stride != 1 or s.name.endswith("down"):
            continue
        key = (s.cin, s.cout, ho, s.name.endswith("conv3"))
        if key in seen:
            continue
        seen.add(key)
        M = a.batch * ho * ho
        x = torch.randn(a.batch, ho, ho, s.cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(s.cout, s.cin, 1, 1, device=dev) * 0.05).to(torch.bfloat16)
        wp = pack_conv_weight(w)
        w2 = w.view(s.cout, s.cin)
        bias = torch.randn(s.cout, device=dev)
        b16 = bias.to(torch.bfloat16)
        res = torch.randn(M, s.cout, device=dev).to(torch.bfloat16) if s.name.endswith("conv3") else None
        outs = [torch.empty(a.batch, ho, ho, s.cout, device=dev, dtype=torch.bfloat16) for _ in range(a.concurrency)]
        cfg, sk = tuning.get(s.name, (0, 0))

        def nat(o, wsc):
            return lambda: conv2d_nhwc(x, wp, bias, kernel=1, residual=None if res is None else res.view(o.shape),
                                       act=1, out=o, workspace=wsc, cfg=cfg, splitk=sk)

        def blas(o, wsc):
            xa = x.view(M, s.cin)
            if res is None:
                return lambda: torch._addmm_activation(b16, xa, w2.t())
            return lambda: torch.relu_(torch.addmm(res, xa, w2.t()).add_(b16))

        tn = autotune._time_multi([nat(o, w_) for o, w_ in zip(outs, ws)], 20)
        tb = autotune._time_multi([blas(o, w_) for o, w_ in zip(outs, ws)], 20)
        print(json.dumps({"layer": s.name, "M": M, "N": s.cout, "K": s.cin, "residual": res is not None,
                          "native_us": round(tn * 1e3, 2), "blas_us": round(tb * 1e3, 2),
                          "concurrency": a.concurrency}), flush=True)


if __name__ == "__main__":
    main()
