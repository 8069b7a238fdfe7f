"""ops.mgemm vs the current route (ops.linear: the tables' native kernels) and hipBLASLt on the
Llama-3-8B decode projections at 64 / 128 / 256 rows (weights L2-cold: a 512 MB scratch fill between
reps would dominate, so the weights of 8 copies rotate instead -- 270 MB+ per set > MALL)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gateup": (28672, 4096), "down": (4096, 14336),
          "lm": (128256, 4096)}


def timeit(fn, reps):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    st.record()
    for i in range(reps):
        fn(i)
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1e3 / reps


FORCE_TILE = False


def main():
    os.environ["MLS_MGEMM"] = "0"  # "route" = the table route the model used before the mgemm route
    from mlmicroservicetemplate_amd import ops

    dev = torch.device("cuda:0")
    rows = [int(r) for r in os.environ.get("ROWS", "64,128,256").split(",")]
    names = os.environ.get("SHAPES", "qkv,o,gateup,down,lm").split(",")
    splits = [int(s) for s in os.environ.get("SPLITS", "0").split(",")]
    # one preallocated fp32 workspace for every call, as the model passes (split-K slabs / counters)
    wsb = torch.zeros(64 << 20, device=dev, dtype=torch.float32)
    for name in names:
        N, K = SHAPES[name]
        copies = max(1, min(8, int(2.5e9 // (N * K * 2))))
        ws = [torch.randn(N, K, device=dev).mul_(K**-0.5).to(torch.bfloat16) for _ in range(copies)]
        act = "silu_mul" if name == "gateup" else "none"
        for M in rows:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            res = None if act == "silu_mul" else torch.randn(M, N, device=dev).to(torch.bfloat16)
            ref = ops.linear(x, ws[0], act=act, residual=res)
            rec = {"shape": name, "M": M, "N": N, "K": K, "copies": copies,
                   "route_us": round(timeit(lambda i: ops.linear(x, ws[i % copies], act=act, residual=res,
                                                                  workspace=wsb, impl="tile" if FORCE_TILE else "auto"), 20), 2),
                   "blas_us": round(timeit(lambda i: ops.linear(x, ws[i % copies], act=act, residual=res, impl="blas"), 20), 2)}
            for s in splits:
                out = ops.mgemm(x, ws[0], act=act, residual=res, splitk=s)
                err = ((out.float() - ref.float()).abs().max() / (ref.float().abs().max() + 1e-6)).item()
                t = timeit(lambda i: ops.mgemm(x, ws[i % copies], act=act, residual=res, splitk=s, workspace=wsb), 20)
                rec[f"mgemm_s{s}_us"] = round(t, 2)
                rec[f"mgemm_s{s}_rel_err_vs_route"] = round(err, 5)
                rec[f"mgemm_s{s}_tb_s"] = round(N * K * 2 / t / 1e6, 2)
            print(json.dumps(rec), flush=True)
        del ws


if __name__ == "__main__":
    main()
