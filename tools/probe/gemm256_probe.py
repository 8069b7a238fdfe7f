"""Large plain GEMMs (BERT-base projections at T = 4096 tokens, Llama prefill shapes): native
conv_gemm tile configs (incl. the 256-wide ones) vs hipBLASLt (torch.mm), alone (c1) and as 4
co-running copies on 4 streams (c4, the engine's regime).  TFLOP/s per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = {"bert_qkv": (4096, 2304, 768), "bert_o": (4096, 768, 768), "bert_ffn1": (4096, 3072, 768),
          "bert_ffn2": (4096, 768, 3072), "llama_qkv_p512": (512, 6144, 4096), "llama_gu_p4096": (4096, 28672, 4096),
          "llama_o_p512": (512, 4096, 4096), "llama_gu_p512": (512, 28672, 4096), "llama_down_p512": (512, 4096, 14336)}
if os.environ.get("SHAPES"):
    SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ["SHAPES"].split(",")}


def timed(fn, conc, iters=20):
    streams = [torch.cuda.Stream() for _ in range(conc)]
    for s in streams:
        with torch.cuda.stream(s):
            fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for s in streams:
        s.wait_event(t0)
    for _ in range(iters):
        for s in streams:
            with torch.cuda.stream(s):
                fn()
    for s in streams:
        ev = torch.cuda.Event()
        ev.record(s)
        torch.cuda.current_stream().wait_event(ev)
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / (iters * conc)  # us per call (amortised)


def main():
    from mlmicroservicetemplate_amd import ops

    dev = torch.device("cuda:0")
    cfgs = [int(c) for c in os.environ.get("CFGS", "1,5,12,27,29,30,31").split(",")]
    ws = torch.empty(64 << 20, device=dev, dtype=torch.float32)
    for name, (M, N, K) in SHAPES.items():
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K**0.5).to(torch.bfloat16)
        flop = 2.0 * M * N * K
        impls = {"hipblaslt": lambda: torch.mm(a, w.t())}
        for c in cfgs:
            impls[f"cfg{c}"] = (lambda c=c: ops.gemm(a, w, workspace=ws, cfg=c, splitk=1))
        ref = a.float() @ w.float().t()
        for c in cfgs:
            out = ops.gemm(a, w, workspace=ws, cfg=c, splitk=1)
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            assert err < 2e-2, (name, c, err)
        for conc in [int(c) for c in os.environ.get("CONC", "1,4").split(",")]:
            for impl, fn in impls.items():
                us = timed(fn, conc)
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "conc": conc, "impl": impl,
                                  "us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
