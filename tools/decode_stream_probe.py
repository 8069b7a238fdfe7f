"""Cold-weight decode GEMM streaming: 32 distinct weight matrices per shape (as the 32 layers of a
decode step), replayed back-to-back in one hipGraph, so every call reads its weights from HBM
(the single-matrix probe is flattered by the 256 MB Infinity Cache).  Skinny kernel variants vs
hipBLASLt; µs per call and HBM TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops.autotune import _time

    dev = torch.device("cuda:0")
    ws = torch.empty(64 << 20, device=dev)
    M = int(os.environ.get("M", "1"))
    if os.environ.get("BLAS_TUNING") == "1":  # hipBLASLt on the shipped TunableOp table
        ops.load_blas_tuning()
    for name, (N, K) in SHAPES.items():
        ws_list = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(32)]
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        d = torch.randn(M, K, device=dev).to(torch.bfloat16)
        r_out = torch.empty_like(x)
        act = "silu_mul" if name == "gate_up" else "none"
        impls = {
            "skinny": lambda: [ops.gemm(x, w, act=act, workspace=ws) for w in ws_list],
            "hipblaslt": lambda: [torch.mm(x, w.t()) for w in ws_list],
        }
        if K == 4096 and name != "o" and M <= 32:
            impls["fused_norm_skinny"] = lambda: [ops.gemm_rmsnorm(x, w, d, r_out, act=act, workspace=ws)
                                                  for w in ws_list]
        if os.environ.get("GEMM_CFGS"):  # native tile configs x split-K factors (ops.gemm cfg / splitk)
            for c in [int(t) for t in os.environ["GEMM_CFGS"].split(",")]:
                for sk in [int(t) for t in os.environ.get("GEMM_SPLITS", "1,2,4,8").split(",")]:
                    impls[f"gemm_c{c}_s{sk}"] = (lambda c=c, sk=sk: [ops.gemm(x, w, act=act, workspace=ws, cfg=c, splitk=sk)
                                                               for w in ws_list])
        lib = ops.lib()

        def variant(fn, no_lds):
            def run():
                lib.mls_skinny_set_variant(no_lds)
                fn()
                lib.mls_skinny_set_variant(0)
            return run

        if hasattr(lib, "mls_skinny_set_variant") and os.environ.get("REG", "0") == "1":
            for k in [k for k in impls if "skinny" in k]:
                impls[k + "_reg"] = variant(impls[k], 1)
        if M <= 4 and os.environ.get("FP8_VARIANTS"):  # W8A8 e4m3 (ops.pack_skinny_fp8): half the bytes
            q_list = [ops.pack_skinny_fp8(w) for w in ws_list]
            for v in [int(t) for t in os.environ["FP8_VARIANTS"].split(",")]:
                if M * K * 2 <= 65536:
                    impls[f"fp8_v{v}"] = (lambda v=v: [ops.skinny_fp8(x, q, sc, N, act=act, variant=v) for q, sc in q_list])
                    if K == 4096 and name != "o":
                        impls[f"fused_norm_fp8_v{v}"] = (
                            lambda v=v: [ops.skinny_fp8(x, q, sc, N, delta=d, resid_out=r_out, norm=True, act=act,
                                                        variant=v) for q, sc in q_list])
        if M <= int(os.environ.get("PACKED_MAX_M", "16")):  # packed 1 KiB-granule weights (ops.pack_skinny), variants of mls_skinny_packed
            wp_list = [ops.pack_skinny(w) for w in ws_list]
            norm_fused = K == 4096 and name != "o"
            for v in [int(t) for t in os.environ.get("PACKED_VARIANTS", "0,1,2,3,4,5").split(",")]:
                impls[f"packed_v{v}"] = (lambda v=v: [ops.skinny_packed(x, wp, N, act=act, variant=v) for wp in wp_list])
                if norm_fused:
                    impls[f"norm_packed_v{v}"] = (
                        lambda v=v: [ops.skinny_packed(x, wp, N, norm=True, act=act, variant=v) for wp in wp_list])
                    impls[f"fused_norm_packed_v{v}"] = (
                        lambda v=v: [ops.skinny_packed(x, wp, N, delta=d, resid_out=r_out, norm=True, act=act, variant=v)
                                     for wp in wp_list])
        for impl, fn in impls.items():
            t = _time(fn, iters=3) * 1e-3 / 32
            print(json.dumps({"shape": name, "M": M, "impl": impl, "us_per_call": round(t * 1e6, 2),
                              "hbm_tb_s": round(N * K * 2 / t / 1e12, 2)}), flush=True)
        del ws_list
        impls.clear()
        wp_list = None
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
