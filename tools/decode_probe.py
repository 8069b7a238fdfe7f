"""Decode-shaped products on one MI355X, graph-timed: the fused RMSNorm+skinny GEMM
(``ops.gemm_rmsnorm``) vs standalone RMSNorm + skinny GEMM, and the plain skinny GEMM against
hipBLASLt, on the Llama-3-8B projection shapes.  One JSON line per (shape, M, impl)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops.autotune import _time

    dev = torch.device("cuda:0")
    ws = torch.empty(64 << 20, device=dev, dtype=torch.float32)
    Ms = [int(m) for m in (sys.argv[1:] or ["1", "4", "8", "16"])]
    for name, (N, K) in SHAPES.items():
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        gain = torch.ones(K, device=dev, dtype=torch.bfloat16)
        act = "silu_mul" if name == "gate_up" else "none"
        for M in Ms:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            d = torch.randn(M, K, device=dev).to(torch.bfloat16)
            r_out = torch.empty_like(x)
            res = {
                "skinny": lambda: ops.gemm(x, w, act=act, workspace=ws),
                "hipblaslt": lambda: torch.mm(x, w.t()),
            }
            if K == 4096:
                res["norm+skinny"] = lambda: ops.gemm(ops.rmsnorm(d, gain, residual=x, residual_out=r_out), w,
                                                      act=act, workspace=ws)
                res["fused_norm_skinny"] = lambda: ops.gemm_rmsnorm(x, w, d, r_out, act=act, workspace=ws)
            for impl, fn in res.items():
                t = _time(fn, iters=50) * 1e-3
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "impl": impl, "us": round(t * 1e6, 2),
                                  "weight_tb_s": round(N * K * 2 / t / 1e12, 2)}), flush=True)
            del x, d, r_out
        del w


if __name__ == "__main__":
    main()
