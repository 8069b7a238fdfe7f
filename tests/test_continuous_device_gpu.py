"""Device-resident continuous batching (models/llama_serving.py ``_iteration_dev``: per-slot state
on the GPU, prefill picks written into the slots, the decode step + X4 + pick as ONE captured
graph, one [2, B] read-back per iteration) against the host-pick path on the same fused model:
identical tokens for staggered greedy / sampled requests, with per-slot and paged KV caches."""
import pytest
import torch

pytestmark = pytest.mark.gpu
CFG = dict(vocab=4096, hidden=512, layers=2, heads=8, kv_heads=2, head_dim=64, intermediate=1024)


def _serve(m, reqs, dev_mode: bool):
    from mlmicroservicetemplate_amd.models.llama_serving import ContinuousLlama

    eng = ContinuousLlama(m)
    eng._want_dev = dev_mode
    # every request queued before the scheduler starts: the admission order (first 4, then one per
    # freed slot) is then a function of the tokens alone, so both modes run the same prefill
    # batches (staggered arrivals: tests/test_continuous_batching.py)
    futs = [eng.submit(ids, gp) for ids, gp in reqs]
    eng.start()
    outs = [f.result(timeout=120) for f in futs]
    eng.stop()
    return outs, eng


@pytest.mark.parametrize("kv_pages", [0, 40])
def test_device_iterations_match_host_picks(kv_pages):
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config(**CFG)
    p = init_llama_shard(cfg, 1, 0, seed=5, device="cuda")
    g = torch.Generator().manual_seed(1)
    reqs = []
    for i in range(11):  # more requests than the 4 slots
        n = int(torch.randint(2, 40, (1,), generator=g))
        ids = torch.randint(3, cfg.vocab - 1, (n,), generator=g).tolist()
        gp = GenParams(max_new_tokens=int(torch.randint(1, 12, (1,), generator=g)), top_k=[1, 8, 1, 40][i % 4],
                       temperature=[1.0, 0.7, 1.0, 1.3][i % 4], seed=100 + i)
        reqs.append((ids, gp))
    res = {}
    for mode in (False, True):
        m = LlamaTP(p, cfg, backend="fused", device="cuda", max_batch=4, max_seq=128, kv_pages=kv_pages)
        res[mode] = _serve(m, reqs, mode)
    (host_out, host_eng), (dev_out, dev_eng) = res[False], res[True]
    assert not host_eng.dev_mode and dev_eng.dev_mode
    assert dev_out == host_out
    # one device -> host copy per iteration that did work (the [2, B] read-back)
    assert 0 < dev_eng.host_reads <= dev_eng.iterations
    assert dev_eng.stats()["active"] == 0
    st = dev_eng.m.serve_state(4)
    assert int(st["active"].sum()) == 0 and int(st["pos"].abs().sum()) == 0  # retired slots reset
