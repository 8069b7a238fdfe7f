"""Debug aid: the /generate service vs the same tiny Llama called directly (one process)."""
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from fastapi.testclient import TestClient

    from mlmicroservicetemplate_amd.api.app import create_app
    from mlmicroservicetemplate_amd.config import Settings
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config(layers=2, head_dim=128, heads=4, kv_heads=1)
    ids = [1, 55, 99, 1000, 7, 8]

    def direct(graphs=True):
        m = LlamaTP(init_llama_shard(cfg, 1, 0, seed=0, device="cuda"), cfg, backend="fused", device="cuda",
                    max_batch=4, max_seq=256)
        m.use_graphs = graphs
        return m.generate(torch.tensor([ids], dtype=torch.int32), torch.tensor([len(ids)], dtype=torch.int32),
                          GenParams(6))[0].tolist(), m

    a, ma = direct()
    print("direct A", a, flush=True)
    y = os.path.join(tempfile.mkdtemp(), "llama.yaml")
    open(y, "w").write("config: tiny\nmax_seq: 256\noverrides:\n  layers: 2\n  head_dim: 128\n  heads: 4\n  kv_heads: 1\n")
    s = Settings.load(env_file=None, environ={}, overrides={"REGISTER": False, "GPUS": 1, "MODEL": "llama",
                                                           "MODEL_CONFIG": y, "MAX_BATCH": 4, "BACKEND": "fused"})
    app = create_app(s)
    with TestClient(app) as c:
        t0 = time.time()
        while c.get("/status").status_code != 200 and time.time() - t0 < 120:
            time.sleep(0.1)
        r = c.post("/generate", json={"input_ids": ids, "max_new_tokens": 6})
        print("service", r.json()["result"]["token_ids"], flush=True)
        sm = app.state.runtime.plugin.model
        for k in ("embed", "l0.qkv", "l0.gate_up", "lm_head", "final_norm"):
            if k in sm.p and k in ma.p:
                print(k, tuple(sm.p[k].shape), tuple(ma.p[k].shape),
                      float((sm.p[k].float() - ma.p[k].float()).abs().max()), flush=True)
        print("service model: backend", sm.backend, "graphs", sm.use_graphs, "max_batch", sm.max_batch,
              "max_seq", sm.max_seq, "cfg", sm.cfg, flush=True)
        out = sm.generate(torch.tensor([ids], dtype=torch.int32), torch.tensor([len(ids)], dtype=torch.int32),
                          GenParams(6))[0].tolist()
        print("service model direct call", out, flush=True)
    b, _ = direct()
    print("direct B", b, flush=True)


if __name__ == "__main__":
    main()
