"""BERT-base B=32 S=128 projections (M = 4096): hipBLASLt (ops.linear impl="blas") vs the native
MFMA GEMM at its best (cfg, split-K), graph-timed per call alone and with 4 copies co-running.
Run once plain and once with PyTorch TunableOp on to see whether the library's default solution
choice leaves time on the table."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mlmicroservicetemplate_amd import ops  # noqa: E402
from mlmicroservicetemplate_amd.ops import autotune  # noqa: E402

dev = torch.device("cuda:0")
M = 4096
SHAPES = {"qkv": (2304, 768, ops.ACT_NONE, False), "o": (768, 768, ops.ACT_NONE, True),
          "ffn1": (3072, 768, ops.ACT_GELU, False), "ffn2": (768, 3072, ops.ACT_NONE, True)}
tag = os.environ.get("PROBE_TAG", "plain")
for name, (N, K, act, resid) in SHAPES.items():
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=dev) * 0.1
    r = torch.randn(M, N, device=dev).to(torch.bfloat16) if resid else None
    for conc in (1, 4):
        outs = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(conc)]
        wss = [torch.empty(4 << 20, device=dev, dtype=torch.float32) for _ in range(conc)]
        # library path as the model uses it: bias (+GELU) epilogue; the residual goes to the LN kernel
        t_blas = autotune._time_multi([lambda: ops.linear(a, w, b, act=act, impl="blas") for _ in range(conc)], 20)
        best = None
        if tag == "plain":
            for cfg in range(1, 19):
                for sk in (1, 2):
                    try:
                        fns = [lambda o=o, ws=ws: ops.gemm(a, w, b, act=act, residual=r, out=o, workspace=ws, cfg=cfg,
                                                           splitk=sk) for o, ws in zip(outs, wss)]
                        t = autotune._time_multi(fns, 20)
                    except Exception:  # config not valid for this shape
                        continue
                    if best is None or t < best[0]:
                        best = (t, cfg, sk)
        rec = {"tag": tag, "shape": name, "M": M, "N": N, "K": K, "concurrency": conc,
               "blas_us": round(t_blas * 1e3, 2), "tflops_blas": round(2 * M * N * K / t_blas / 1e9, 1)}
        if best:
            rec.update({"native_us": round(best[0] * 1e3, 2), "native_cfg": best[1], "native_splitk": best[2],
                        "tflops_native": round(2 * M * N * K / best[0] / 1e9, 1)})
        print(json.dumps(rec), flush=True)
