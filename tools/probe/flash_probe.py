"""Llama-shaped prefill attention (causal, GQA 32 / 8 heads, D = 128) alone: time per call of
ops.flash_attention at the given batches, checked against an fp32 PyTorch reference.

    python3 tools/probe/flash_probe.py --batches 1 8 --seq 512 [--iters 50]
Prints one JSON line per batch."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def reference(qkv, B, S, hq, hkv, D):
    q, k, v = qkv.float().split([hq * D, hkv * D, hkv * D], dim=1)
    q = q.view(B, S, hq, D).transpose(1, 2)
    k = k.view(B, S, hkv, D).transpose(1, 2).repeat_interleave(hq // hkv, dim=1)
    v = v.view(B, S, hkv, D).transpose(1, 2).repeat_interleave(hq // hkv, dim=1)
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
    return o.transpose(1, 2).reshape(B * S, hq * D)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    from mlmicroservicetemplate_amd import ops

    dev = torch.device("cuda:0")
    D = 128
    for B in a.batches:
        g = torch.Generator(device="cpu").manual_seed(B)
        qkv = torch.randn(B * a.seq, (a.hq + 2 * a.hkv) * D, generator=g).to(torch.bfloat16).to(dev)
        lens = torch.full((B,), a.seq, dtype=torch.int32, device=dev)
        out = ops.flash_attention(qkv, B, a.seq, a.hq, a.hkv, D, kv_lens=lens, causal=True)
        ref = reference(qkv, B, a.seq, a.hq, a.hkv, D)
        err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        for _ in range(5):
            ops.flash_attention(qkv, B, a.seq, a.hq, a.hkv, D, kv_lens=lens, causal=True, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            ops.flash_attention(qkv, B, a.seq, a.hq, a.hkv, D, kv_lens=lens, causal=True, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        flop = 4.0 * B * a.hq * a.seq * a.seq * D / 2  # causal half
        print(json.dumps({"probe": "flash_llama", "tag": a.tag, "batch": B, "seq": a.seq, "us": round(us, 2),
                          "tflops": round(flop / us / 1e6, 1), "rel_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
