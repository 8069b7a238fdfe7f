"""1x1 stride-1 ResNet-50 convs (bs=32) on the persistent GEMM tile kernel (csrc/gemm_tile.hip:
act(A . W^T + bias (+ residual)), A = the NHWC activation as [M][Cin], W = the packed [Cout][Cin]
weight) vs the shipped conv_gemm table entry, per tile cfg x in-launch split-K, alone (c1) and with
4 copies co-running on their own streams (c4).  One JSON line per (layer, impl, concurrency)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.models.resnet import conv_shapes  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune, conv2d_nhwc, pack_conv_weight  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--cfgs", type=int, nargs="*", default=[1, 2, 3, 5, 21])
    ap.add_argument("--splitk", type=int, nargs="*", default=[1, 2, 4])
    ap.add_argument("--conc", type=int, nargs="*", default=[1, 4])
    ap.add_argument("--layers", nargs="*", default=None, help="layer-name prefixes (default: layer2..4)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tuning = autotune.load_tuning("resnet50", a.batch)
    C = max(a.conc)
    ws = [torch.zeros(64 << 20, device=dev, dtype=torch.float32) for _ in range(C)]
    prefixes = a.layers or ["layer2", "layer3", "layer4"]
    seen = set()
    torch.manual_seed(0)
    for s, hin, ho in conv_shapes():
        if s.k != 1 or s.stride != 1 or s.name.endswith("down") or not any(s.name.startswith(p) for p in prefixes):
            continue
        conv3 = s.name.endswith("conv3")
        key = (s.cin, s.cout, ho, conv3)
        if key in seen:
            continue
        seen.add(key)
        M = a.batch * ho * ho
        xs = [(torch.rand(a.batch, ho, ho, s.cin, device=dev) * 2 - 1).to(torch.bfloat16) for _ in range(C)]
        w = ((torch.rand(s.cout, s.cin, 1, 1, device=dev) * 2 - 1) / s.cin ** 0.5).to(torch.bfloat16)
        wp = pack_conv_weight(w)
        w2 = wp.view(s.cout, s.cin)
        bias = torch.randn(s.cout, device=dev) * 0.1
        res = (torch.rand(M, s.cout, device=dev) * 2 - 1).to(torch.bfloat16) if conv3 else None
        outs = [torch.empty(a.batch, ho, ho, s.cout, device=dev, dtype=torch.bfloat16) for _ in range(C)]
        ref = torch.relu(xs[0].view(M, s.cin).float() @ w2.float().T + bias + (res.float() if conv3 else 0))
        cfg, sk = tuning.get(s.name, (0, 0))

        def nat(i):
            return lambda: conv2d_nhwc(xs[i], wp, bias, kernel=1, residual=None if res is None else res.view(outs[i].shape),
                                       act=1, out=outs[i], workspace=ws[i], cfg=cfg, splitk=sk)

        impls = [(f"conv_cfg{cfg}s{sk}", nat)]
        for c in a.cfgs:
            for k in a.splitk:
                def tile(i, c=c, k=k):
                    return lambda: ops.gemm_tile(xs[i].view(M, s.cin), w2, bias, act=ops.ACT_RELU, residual=res,
                                                 out=outs[i].view(M, s.cout), cfg=c, splitk=k, workspace=ws[i])
                impls.append((f"tile{c}s{k}", tile))
        for name, mk in impls:
            try:
                mk(0)()
                torch.cuda.synchronize()
            except Exception as e:  # unsupported split for this K
                print(json.dumps({"layer": s.name, "impl": name, "error": str(e)[:160]}), flush=True)
                continue
            err = ((outs[0].view(M, s.cout).float() - ref).abs().max() / ref.abs().max()).item()
            for c in a.conc:
                t = autotune._time_multi([mk(i) for i in range(c)], 20)
                print(json.dumps({"layer": s.name, "M": M, "N": s.cout, "K": s.cin, "residual": conv3, "impl": name,
                                  "conc": c, "us": round(t * 1e3, 2),
                                  "tflops": round(2.0 * M * s.cout * s.cin / (t * 1e-3) / 1e12, 1),
                                  "rel_err": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
