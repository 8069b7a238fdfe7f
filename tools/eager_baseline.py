"""Comparison baseline (b) of SURVEY.md §6: stock PyTorch-ROCm (MIOpen/hipBLASLt) ResNet-50.

Measures ms per bs=32 forward (uint8 images -> normalise -> logits -> softmax -> top-5) in
bf16 channels-last, eager and hipGraph-captured, on the same random weights the fused path
uses.  Prints one JSON line per variant.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mlmicroservicetemplate_amd.models.resnet import (  # noqa: E402
    ResNet50Eager,
    init_resnet50,
    resnet50_flops_per_image,
    resnet50_reference,
)


def timeit(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    p = torch.cuda.get_device_properties(dev)
    print(json.dumps({"device": p.name, "gcn": getattr(p, "gcnArchName", "?"), "cus": p.multi_processor_count,
                      "mem_gb": p.total_memory / 2**30, "torch": torch.__version__, "hip": torch.version.hip}))
    params = init_resnet50(0)
    imgs = torch.randint(0, 256, (args.batch, 224, 224, 3), dtype=torch.uint8, device=dev)
    gflop = resnet50_flops_per_image() * args.batch / 1e9
    for fold in (False, True):
        model = ResNet50Eager(params, dev, fold=fold)

        def step():
            logits = model(imgs)
            probs = torch.softmax(logits.float(), dim=-1)
            return torch.topk(probs, 5, dim=-1)

        with torch.no_grad():
            ref = resnet50_reference({k: v.to(dev) for k, v in params.items()}, imgs)
            out = model(imgs).float()
            err = (out - ref).abs().max().item() / ref.abs().max().item()
            ms = timeit(step, args.steps, args.warmup)
            # hipGraph capture of the eager path
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    step()
            torch.cuda.current_stream().wait_stream(s)
            with torch.cuda.graph(g):
                step()
            ms_g = timeit(g.replay, args.steps, args.warmup)
        for name, t in (("eager", ms), ("eager+hipgraph", ms_g)):
            print(json.dumps({"variant": name, "bn_folded": fold, "batch": args.batch, "ms_per_batch": round(t, 4),
                              "img_per_s": round(args.batch / t * 1e3, 1), "tflops": round(gflop / t, 2),
                              "rel_err_vs_fp32": err}))


if __name__ == "__main__":
    main()
