"""Continuous batching for /generate (models/llama_serving.py) on CPU: sequences that join and
leave the running batch at arbitrary steps produce exactly what a batch-of-one generate() gives,
more requests than KV slots queue, EOS retires a sequence early."""
import time

import pytest
import torch

from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config
from mlmicroservicetemplate_amd.models.llama_serving import ContinuousLlama, EngineFull

CFG = dict(vocab=2048, hidden=256, layers=2, heads=8, kv_heads=4, head_dim=32, intermediate=512)


@pytest.fixture(scope="module")
def params():
    torch.set_num_threads(1)
    cfg = tiny_config(**CFG)
    return cfg, init_llama_shard(cfg, 1, 0, seed=4)


def _single(cfg, p, ids, gp):
    m = LlamaTP(p, cfg, max_batch=1, max_seq=96)
    return m.generate(torch.tensor([ids]), torch.tensor([len(ids)]), gp)[0].tolist()


def test_staggered_requests_match_batch_of_one(params):
    cfg, p = params
    m = LlamaTP(p, cfg, max_batch=3, max_seq=96)
    eng = ContinuousLlama(m).start()
    g = torch.Generator().manual_seed(0)
    reqs = []
    for i in range(7):  # more requests than the 3 slots
        n = int(torch.randint(2, 20, (1,), generator=g))
        ids = torch.randint(3, 2000, (n,), generator=g).tolist()
        gp = GenParams(max_new_tokens=int(torch.randint(1, 9, (1,), generator=g)), top_k=[1, 5][i % 2],
                       temperature=0.7, seed=i)
        reqs.append((ids, gp))
    futs = []
    for ids, gp in reqs:
        futs.append(eng.submit(ids, gp))
        time.sleep(0.01)  # arrive while others are mid-decode
    outs = [f.result(timeout=60) for f in futs]
    eng.stop()
    eos = set(cfg.eos_ids)
    for (ids, gp), got in zip(reqs, outs):
        want = _single(cfg, p, ids, gp)
        cut = next((i + 1 for i, t in enumerate(want) if t in eos), len(want))
        assert got == want[:cut], (ids, gp, got, want)
    assert eng.stats()["active"] == 0 and eng.iterations > 0


def test_eos_retires_and_slot_is_reused(params):
    cfg, p = params
    m = LlamaTP(p, cfg, max_batch=1, max_seq=96)
    ids = [5, 6, 7, 8]
    first = _single(cfg, p, ids, GenParams(6))
    # make the second generated token an end-of-sequence id
    m.cfg.eos_ids = (first[1],)
    eng = ContinuousLlama(m).start()
    a = eng.submit(ids, GenParams(6)).result(timeout=60)
    b = eng.submit([9, 10], GenParams(3)).result(timeout=60)  # the freed slot serves the next request
    eng.stop()
    assert a == first[: first.index(first[1]) + 1] and len(b) >= 1


def test_queue_bound_and_validation(params):
    cfg, p = params
    m = LlamaTP(p, cfg, max_batch=1, max_seq=32)
    eng = ContinuousLlama(m, max_queue=1)  # not started: nothing drains the queue
    eng.submit([1, 2], GenParams(2))
    with pytest.raises(EngineFull):
        eng.submit([1, 2], GenParams(2))
    with pytest.raises(ValueError):
        eng.submit([1] * 30, GenParams(8))
    with pytest.raises(ValueError):
        eng.submit([], GenParams(1))


def test_vectorised_picks_match_pick_token():
    """ContinuousLlama._pick_rows == LlamaTP.pick_token row by row: greedy rows (ties resolve to
    the first maximum) in one argmax / gather, sampled rows on the seeded per-row path."""
    g = torch.Generator().manual_seed(0)
    cv = torch.randn(6, 16, generator=g)
    cv[2, 3] = cv[2, 9] = cv[2].max() + 1.0  # a tie
    ci = torch.randint(0, 1000, (6, 16), generator=g)
    rows = [(0, GenParams(top_k=1), 0), (2, GenParams(top_k=1), 3), (5, GenParams(8, top_k=5, seed=2), 4),
            (4, GenParams(top_k=1), 1), (1, GenParams(8, top_k=3, temperature=0.5, seed=9), 0)]
    eng = object.__new__(ContinuousLlama)
    eng.m = LlamaTP  # pick_token is a staticmethod
    got = eng._pick_rows(cv, ci, rows)
    want = [LlamaTP.pick_token(cv[r], ci[r], gp, step) for r, gp, step in rows]
    assert got == want
    assert got[1] == int(ci[2, 3])
