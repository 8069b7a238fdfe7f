"""Greedy generate of a tiny Llama on the GPU: reference backend vs fused (eager steps) vs fused
(hipGraph decode) -- the three must agree token for token (debug aid + GPU test helper)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(S=6, n=8, layers=2):
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config(layers=layers, head_dim=128, heads=4, kv_heads=1)
    p = init_llama_shard(cfg, 1, 0, seed=0, device="cuda")
    ids = torch.tensor([[(37 * i + 11) % 2000 + 3 for i in range(S)]], device="cuda")
    lens = torch.tensor([S], device="cuda")
    out = {}
    for name, backend, graphs in (("reference", "reference", False), ("fused_eager", "fused", False),
                                  ("fused_graph", "fused", True)):
        m = LlamaTP(p, cfg, backend=backend, device="cuda", max_batch=4, max_seq=256)
        m.use_graphs = graphs
        out[name] = m.generate(ids, lens, GenParams(n))[0].tolist()
    return out


if __name__ == "__main__":
    for S in (6, 16, 40):
        print(S, run(S))
