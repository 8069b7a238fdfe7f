"""Plain-GEMM throughput probe: every ops.gemm config (and the heuristic) vs torch.matmul (hipBLASLt)
on the transformer shapes of configs 3 and 5 (graph-timed, so launch cost is excluded).
One JSON line per (shape, impl)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (M, N, K)
    "llama_qkv": (4096, 6144, 4096), "llama_o": (4096, 4096, 4096), "llama_gateup": (4096, 28672, 4096),
    "llama_down": (4096, 4096, 14336), "bert_qkv": (4096, 2304, 768), "bert_ffn1": (4096, 3072, 768),
    "bert_ffn2": (4096, 768, 3072), "dec16_qkv": (16, 6144, 4096), "dec16_gateup": (16, 28672, 4096),
    "dec1_down": (1, 4096, 14336), "dec8_down": (8, 4096, 14336), "dec32_gateup": (32, 28672, 4096),
    "bert128_qkv": (128, 2304, 768), "bert128_ffn1": (128, 3072, 768), "bert128_ffn2": (128, 768, 3072),
    "bert128_o": (128, 768, 768), "bert32_o": (32, 768, 768), "bert32_ffn1": (32, 3072, 768),
    "bert32_ffn2": (32, 768, 3072), "bert1024_qkv": (1024, 2304, 768), "bert1024_ffn2": (1024, 768, 3072),
    "m64_qkv": (64, 6144, 4096), "m256_gateup": (256, 28672, 4096),
    "dec256_qkv": (256, 6144, 4096), "dec256_o": (256, 4096, 4096), "dec256_down": (256, 4096, 14336),
    "dec256_lm": (256, 128256, 4096),
}


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops.autotune import _time

    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=list(SHAPES))
    ap.add_argument("--cfgs", type=int, nargs="*", default=list(range(0, 13)))
    ap.add_argument("--splitk", type=int, nargs="*", default=[1])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ws = torch.empty(64 << 20, device=dev, dtype=torch.float32)
    for name in a.shapes:
        M, N, K = SHAPES[name]
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        flop = 2.0 * M * N * K
        byt = 2.0 * (M * K + N * K + M * N)
        res = []
        t = _time(lambda: torch.matmul(x, w.T), iters=20)
        res.append(("torch", 0, t))
        for cfg in a.cfgs:
            for sk in a.splitk:
                try:
                    t = _time(lambda: ops.gemm(x, w, workspace=ws, cfg=cfg, splitk=0 if cfg == 0 else sk), iters=20)
                except Exception as e:  # unsupported combination
                    continue
                res.append(("heuristic" if cfg == 0 else f"cfg{cfg}", sk, t))
        for impl, sk, t_ms in res:
            t = t_ms * 1e-3
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "impl": impl, "splitk": sk,
                              "us": round(t * 1e6, 1), "tflops": round(flop / t / 1e12, 1),
                              "tb_s": round(byt / t / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
