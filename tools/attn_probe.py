"""Decode-attention launch time (graph-timed) over batch, context length and split size, plain and
rope/append mode, Llama-3-8B head geometry (32 q heads, 8 kv heads, D=128, TP=1)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops import reference as R
    from mlmicroservicetemplate_amd.ops.autotune import _time

    dev = torch.device("cuda:0")
    Hq, Hkv, D, max_len = 32, 8, 128, 2048
    cos, sin = R.rope_tables(max_len, D, 500000.0, dev)
    for B in (1, 8, 32):
        kc = torch.randn(B, max_len, Hkv, D, device=dev).to(torch.bfloat16)
        vc = torch.randn_like(kc)
        qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
        ws = torch.empty(B * Hq * (max_len // 16) * (D + 2), device=dev)
        cnt = torch.zeros(B * Hkv, device=dev, dtype=torch.int32)
        for L in (129, 1024, 2048):
            lens = torch.full((B,), L, device=dev, dtype=torch.int32)
            pos = lens - 1
            hint = max(256, 1 << (L - 1).bit_length())
            for chunk in (32, 64, 128):
                for rope, ml in ((False, None), (True, None), (True, hint)):
                    kw = dict(positions=pos, cos=cos, sin=sin) if rope else {}
                    t = _time(lambda: ops.decode_attention(qkv, kc, vc, lens, Hq, Hkv, D, chunk=chunk, workspace=ws,
                                                           counters=cnt, max_len=ml, **kw), iters=20)
                    kv_bytes = B * L * Hkv * D * 2 * 2
                    print(json.dumps({"B": B, "L": L, "chunk": chunk, "rope": rope, "max_len": ml or max_len,
                                      "us": round(t * 1e3, 2),
                                      "kv_tb_s": round(kv_bytes / (t * 1e-3) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
