"""X4 on device (ops.decode_pick, csrc/decode_pick.hip) against the host rule
(LlamaTP.pick_token): the merged candidates of every TP rank -> the next token per row (greedy or
seeded top-k sampling), with the decode step's static inputs advanced in place; and the fused
Llama's device-resident decode loop against the host-picked loop."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_decode_pick_matches_host_rule():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP

    torch.manual_seed(0)
    tp, B, k = 4, 6, 8
    cv = torch.randn(tp, B, k) * 3
    cv[1, 2, 3] = float("-inf")  # a padded-vocab candidate
    cv[2, 4, :] = cv[0, 4, 0]  # ties: the first candidate in rank-major order must win
    ci = torch.randint(0, 128256, (tp, B, k), dtype=torch.int32)
    params = [GenParams(top_k=1), GenParams(top_k=5, temperature=0.7, seed=11), GenParams(top_k=32, temperature=1.3, seed=5),
              GenParams(top_k=1), GenParams(top_k=3, temperature=0.01, seed=2), GenParams(top_k=8, seed=123456789012)]
    steps = torch.tensor([0, 3, 7, 1, 0, 42], dtype=torch.int32)
    tok = torch.zeros(B, dtype=torch.int32, device=DEV)
    pos = torch.arange(B, dtype=torch.int32, device=DEV) * 10
    lens = pos + 1
    step = steps.to(DEV)
    hist = torch.full((B, 64), -1, dtype=torch.int32, device=DEV)
    ops.decode_pick(cv.to(DEV), ci.to(DEV), tok, pos, lens, step,
                    topk=torch.tensor([g.top_k for g in params], dtype=torch.int32, device=DEV),
                    temp=torch.tensor([g.temperature for g in params], dtype=torch.float32, device=DEV),
                    seed=torch.tensor([g.seed for g in params], dtype=torch.int64, device=DEV), hist=hist)
    flat_v = cv.permute(1, 0, 2).reshape(B, -1)
    flat_i = ci.permute(1, 0, 2).reshape(B, -1)
    want = [LlamaTP.pick_token(flat_v[b], flat_i[b], params[b], int(steps[b])) for b in range(B)]
    assert tok.cpu().tolist() == want
    assert pos.cpu().tolist() == [10 * b + 1 for b in range(B)] and lens.cpu().tolist() == [10 * b + 2 for b in range(B)]
    assert step.cpu().tolist() == (steps + 1).tolist()
    h = hist.cpu()
    assert [int(h[b, steps[b]]) for b in range(B)] == want


def test_fused_generate_device_loop_matches_host_loop(monkeypatch):
    """Same tokens from the device-resident decode loop (graph replays that pick on device, one
    host copy at the end) as from the host-picked loop, greedy and sampled."""
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config(layers=2, hidden=512, heads=8, kv_heads=2, head_dim=128, intermediate=1024)
    m = LlamaTP(init_llama_shard(cfg, 1, 0, seed=3, device=DEV), cfg, backend="fused", device=DEV, max_batch=4,
                max_seq=256)
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(3, cfg.vocab - 1, (3, 24), generator=g)
    lens = torch.tensor([24, 11, 3])
    for gp in (GenParams(max_new_tokens=12), GenParams(max_new_tokens=12, top_k=8, temperature=0.8, seed=9)):
        k = max(1, min(gp.top_k, m.top_k_max))
        assert m._device_loop_ok(3, k)
        calls = []
        orig = torch.Tensor.cpu

        def counting_cpu(self, *a, **kw):
            if self.is_cuda:
                calls.append(tuple(self.shape))
            return orig(self, *a, **kw)

        monkeypatch.setattr(torch.Tensor, "cpu", counting_cpu)
        dev_out = m.generate(ids, lens, gp)
        monkeypatch.setattr(torch.Tensor, "cpu", orig)
        assert calls == [(3, gp.max_new_tokens)], f"host round trips inside the decode loop: {calls}"
        monkeypatch.setenv("MLS_DEVICE_PICK", "0")
        host_out = m.generate(ids, lens, gp)
        monkeypatch.delenv("MLS_DEVICE_PICK")
        assert torch.equal(dev_out.to(torch.int32), host_out.to(torch.int32)), (dev_out, host_out)
