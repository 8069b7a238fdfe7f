"""Large-M GEMM probe: ops.gemm_tile (csrc/gemm_tile.hip) per tile cfg vs torch.matmul (hipBLASLt)
on the BERT / Llama prefill projection shapes -- numerics (vs fp32) and graph-timed throughput,
alone (c1) and with 4 independent copies co-running on their own streams (c4, how the serving
engine runs them).  One JSON line per (shape, impl, concurrency).  Random [-1, 1)-scale operands
(never zero-filled: cdna_hip_programming.md §5.4 rule 25)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (M, N, K, act)
    "bert32_qkv": (4096, 2304, 768, "none"), "bert32_o": (4096, 768, 768, "none"),
    "bert32_ffn1": (4096, 3072, 768, "gelu"), "bert32_ffn2": (4096, 768, 3072, "none"),
    "bert64_qkv": (8192, 2304, 768, "none"), "bert64_o": (8192, 768, 768, "none"),
    "bert64_ffn1": (8192, 3072, 768, "gelu"), "bert64_ffn2": (8192, 768, 3072, "none"),
    "bert128_qkv": (16384, 2304, 768, "none"), "bert128_o": (16384, 768, 768, "none"),
    "bert128_ffn1": (16384, 3072, 768, "gelu"), "bert128_ffn2": (16384, 768, 3072, "none"),
    "llama_qkv": (4096, 6144, 4096, "none"), "llama_o": (4096, 4096, 4096, "none"),
    "llama_gateup": (4096, 28672, 4096, "silu_mul"), "llama_down": (4096, 4096, 14336, "none"),
    "llama16k_gateup": (16384, 28672, 4096, "silu_mul"), "sq8k": (8192, 8192, 8192, "none"),
    "tp8_qkv": (16384, 768, 4096, "none"), "tp8_gateup": (16384, 3584, 4096, "silu_mul"),
    "tp8_down": (16384, 4096, 1792, "none"), "tp8_o": (16384, 4096, 512, "none"),
    # Llama-3-8B prefill of one 512-token prompt (B=1 x 512 rows)
    "llama512_qkv": (512, 6144, 4096, "none"), "llama512_o": (512, 4096, 4096, "none"),
    "llama512_gateup": (512, 28672, 4096, "silu_mul"), "llama512_down": (512, 4096, 14336, "none"),
    # Llama-3-8B decode step of 256 serving slots (M = 256 rows)
    "dec256_qkv": (256, 6144, 4096, "none"), "dec256_o": (256, 4096, 4096, "none"),
    "dec256_gateup": (256, 28672, 4096, "silu_mul"), "dec256_down": (256, 4096, 14336, "none"),
    "dec256_lm": (256, 128256, 4096, "none"),
    # serving prefill: 256 admitted 128-token prompts in one batch (M = 32768 rows)
    "llama32k_qkv": (32768, 6144, 4096, "none"), "llama32k_o": (32768, 4096, 4096, "none"),
    "llama32k_gateup": (32768, 28672, 4096, "silu_mul"), "llama32k_down": (32768, 4096, 14336, "none"),
}


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops.autotune import _time_multi

    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=list(SHAPES))
    ap.add_argument("--cfgs", type=int, nargs="*", default=[0, 1, 2, 3, 4, 5])
    ap.add_argument("--conc", type=int, nargs="*", default=[1, 4])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splitk", type=int, nargs="*", default=[1], help="K splits per tile cfg (in-launch combine)")
    ap.add_argument("--ablate", type=int, nargs="*", default=[],
                    help="timing-only ablations per cfg (csrc/gemm_tile.hip GT_ABL_*: 1 = no loads, 2 = no stores)")
    ap.add_argument("--stamps", type=int, nargs="*", default=[],
                    help="stamped builds (cfg 13 = cfg 1, 14 = cfg 2): per-block phase cycles of the first tile")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for name in a.shapes:
        M, N, K, act = SHAPES[name]
        code = {"none": ops.ACT_NONE, "gelu": ops.ACT_GELU, "silu_mul": ops.ACT_SILU_MUL}[act]
        xs = [(torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16) for _ in range(max(a.conc))]
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev) * 0.1
        flop = 2.0 * M * N * K
        # fp32 reference on a row slice (the full fp32 product of the big shapes is slow)
        rows = slice(0, min(M, 1024))
        ref = xs[0][rows].float() @ w.float().T + bias
        if code == ops.ACT_GELU:
            ref = torch.nn.functional.gelu(ref)
        elif code == ops.ACT_SILU_MUL:
            g, u = ref.view(ref.shape[0], N // 16, 2, 8).unbind(2)
            ref = (torch.nn.functional.silu(g) * u).reshape(ref.shape[0], N // 2)

        def blas(x):
            if code == ops.ACT_GELU:
                return torch._addmm_activation(bias.to(torch.bfloat16), x, w.t(), use_gelu=True)
            y = torch.addmm(bias.to(torch.bfloat16), x, w.t())
            return ops.silu_mul_interleaved(y) if code == ops.ACT_SILU_MUL else y

        for scfg in a.stamps:
            for ab in [0] + a.ablate:
                r = stamp_run(ops, xs[0], w, bias, code if code != ops.ACT_SILU_MUL else ops.ACT_NONE,
                              scfg | (ab << 8), name)
                print(json.dumps(dict(r, ablate=ab)), flush=True)
        impls = [("hipblaslt", blas, None)] if a.cfgs else []
        ws = torch.zeros(64 << 20, device=dev, dtype=torch.float32)
        for cfg in a.cfgs:
            for sk in a.splitk:
                tag = f"tile{cfg}" + (f"s{sk}" if sk > 1 else "")
                impls.append((tag, (lambda x, c=cfg, k=sk: ops.gemm_tile(x, w, bias, act=code, cfg=c, splitk=k,
                                                                         workspace=ws)), cfg))
            for ab in a.ablate:
                impls.append((f"tile{cfg}ab{ab}", (lambda x, c=cfg | (ab << 8): ops.gemm_tile(x, w, bias, act=code, cfg=c)),
                              cfg))
        for impl, fn, cfg in impls:
            try:
                y = fn(xs[0])
                torch.cuda.synchronize()
            except Exception as e:
                print(json.dumps({"shape": name, "impl": impl, "error": str(e)[:200]}), flush=True)
                continue
            err = ((y[rows].float() - ref).abs().max() / ref.abs().max()).item()
            for c in a.conc:
                t = _time_multi([lambda i=i: fn(xs[i]) for i in range(c)], iters=a.iters) * 1e-3
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "act": act, "impl": impl, "conc": c,
                                  "us": round(t * 1e6, 1), "tflops": round(flop / t / 1e12, 1),
                                  "rel_err": round(err, 5),
                                  "pick": ops.lib().mls_gemm_tile_pick(M, N) if cfg == 0 else cfg}), flush=True)


def stamp_run(ops, x, w, bias, code, cfg, name):
    """One stamped launch (after a warm one): medians over blocks of the first tile's phases in shader
    cycles -- prologue (first k-step landed), per k-step, epilogue issue, store drain -- plus the
    clock from s_memtime vs the 100 MHz s_memrealtime."""
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    buf = torch.zeros(4096, 8, device=x.device, dtype=torch.int64)
    for _ in range(2):
        rc = ops.lib().mls_gemm_tile(x.data_ptr(), w.data_ptr(), bias.data_ptr(), buf.data_ptr(), out.data_ptr(), M, N,
                                     K, code, N, N, cfg, 0, 1, None, 0, None, 0, ops.stream_ptr(x.device))
        ops.check(rc, "mls_gemm_tile")
    torch.cuda.synchronize()
    t = buf[buf[:, 7] > 0].cpu().double()
    nk = K // 64
    med = lambda v: round(float(v.median()), 1)
    span_rt = (t[:, 6].max() - t[:, 5].min()) / 100.0  # us at 100 MHz
    ghz = float(((t[:, 4] - t[:, 0]).sum() / ((t[:, 6] - t[:, 5]).sum() / 100e6)) / 1e9)
    return {"shape": name, "stamp_cfg": cfg, "blocks": int(t.shape[0]), "tiles_per_block_max": int(t[:, 7].max()),
            "clock_ghz": round(ghz, 3), "span_us": round(float(span_rt), 1),
            "start_skew_us": round(float((t[:, 5].max() - t[:, 5].min()) / 100.0), 2),
            "prologue_cyc": med(t[:, 1] - t[:, 0]), "kstep_cyc": med((t[:, 2] - t[:, 1]) / max(1, nk - 1)),
            "epilogue_cyc": med(t[:, 3] - t[:, 2]), "drain_cyc": med(t[:, 4] - t[:, 3]),
            "total_cyc": med(t[:, 4] - t[:, 0]), "ideal_kstep_cyc": None}


if __name__ == "__main__":
    main()
