"""LayerNorm-folding GEMM timing: the BERT projections at T tokens on the plain tile kernels (cfg 15 =
256x256 PIPE, 16 = 256x128 PIPE) vs the folding forms (fold / residual-LN / + row statistics)."""
import json
import sys

import torch

from mlmicroservicetemplate_amd import ops

DEV = "cuda:0"


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


H, I = 768, 3072
for T in [int(t) for t in (sys.argv[1:] or ["16384", "4096"])]:
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(T, H, device=DEV, generator=g).to(torch.bfloat16)
    f = torch.randn(T, I, device=DEV, generator=g).to(torch.bfloat16)
    pin = torch.ones(T * H // 64, device=DEV)
    pout = torch.empty(T * H // 64, device=DEV)
    gam = torch.ones(H, device=DEV)
    for name, N, K, a in (("qkv", 3 * H, H, x), ("o", H, H, x), ("ffn1", I, H, x), ("ffn2", H, I, f)):
        w = (torch.randn(N, K, device=DEV, generator=g) / K**0.5).to(torch.bfloat16)
        b = torch.zeros(N, device=DEV)
        c = torch.zeros(N, device=DEV)
        act = "gelu" if name == "ffn1" else "none"
        r = {}
        for cfg in (15, 16):
            if name in ("o", "ffn2"):
                r[f"plain{cfg}"] = timeit(lambda: ops.gemm_tile(a, w, b, residual=x, cfg=cfg))
            else:
                r[f"plain{cfg}"] = timeit(lambda: ops.gemm_tile(a, w, b, act=act, cfg=cfg))
        for cfg in (15, 16, 5):
            if name in ("o", "ffn2"):
                r[f"res{cfg}"] = timeit(lambda: ops.gemm_tile_ln(a, w, b, residual=x, cfg=cfg))
                r[f"resln{cfg}"] = timeit(lambda: ops.gemm_tile_ln(a, w, b, residual=x, ln_part=pin, ln_g=gam, cfg=cfg))
                r[f"resln_stats{cfg}"] = timeit(lambda: ops.gemm_tile_ln(a, w, b, residual=x, ln_part=pin, ln_g=gam,
                                                                      stats_part=pout, cfg=cfg))
            else:
                r[f"fold{cfg}"] = timeit(lambda: ops.gemm_tile_ln(a, w, b, act=act, fold_c=c, ln_part=pin, cfg=cfg))
        print(json.dumps({"T": T, "proj": name, **{k: round(v, 1) for k, v in r.items()}}), flush=True)
