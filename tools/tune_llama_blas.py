"""Offline PyTorch TunableOp search for the Llama-3-8B projection GEMMs that decode runs on
hipBLASLt (batches above the packed skinny kernels' 24 rows: continuous batching with 32 / 64 /
128 slots) and for the LM head.  Writes the winning solutions to PYTORCH_TUNABLEOP_FILENAME
(append them to ops/tuned/tunableop_gfx950.csv; tuning stays off at run time -- lookup only).

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=out.csv \\
        python tools/tune_llama_blas.py --m 32 64 128
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (N, K) of the TP=1 projections; gate_up is the interleaved [2 x 14336, 4096] matrix
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[32, 64, 128])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    args = ap.parse_args()
    assert torch.cuda.tunable.is_enabled() and torch.cuda.tunable.tuning_is_enabled(), "set PYTORCH_TUNABLEOP_*"
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops.autotune import _time

    dev = torch.device("cuda:0")
    for name in args.shapes:
        N, K = SHAPES[name]
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        for M in args.m:
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            t0 = time.time()
            torch.mm(a, w.t())
            torch.cuda.synchronize()
            print(f"tuned {name} M={M} N={N} K={K} in {time.time() - t0:.1f}s", flush=True)
            if name == "lm_head":  # 1 GB of weights: cold in the 256 MB Infinity Cache on every call
                ws = torch.empty(64 << 20, device=dev)
                for impl, fn in (("hipblaslt_tuned", lambda: torch.mm(a, w.t())),
                                 ("ops.gemm", lambda: ops.gemm(a, w, workspace=ws))):
                    us = _time(fn, iters=10) * 1e3
                    print(json.dumps({"shape": name, "M": M, "impl": impl, "us": round(us, 1),
                                      "hbm_tb_s": round(N * K * 2 / us / 1e6, 2)}), flush=True)
        del w
    return 0  # TunableOp writes PYTORCH_TUNABLEOP_FILENAME itself when the process exits


if __name__ == "__main__":
    sys.exit(main())
