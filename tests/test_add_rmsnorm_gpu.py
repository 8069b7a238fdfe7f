"""ops.linear_add_rmsnorm (conv_gemm.hip mls_gemm_slabs + norm_ops.hip mls_splitk_add_rmsnorm): a
split-K projection reduced together with the residual add + RMSNorm after it must equal ops.linear
followed by ops.rmsnorm(..., residual_out=...) bit for bit -- the op alone and inside the Llama
forward above 24 tokens (o_proj / down_proj)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(64, 4096, 4096), (32, 4096, 14336), (200, 2048, 2048), (33, 4096, 3072)])
def test_matches_linear_then_rmsnorm(M, N, K):
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(M + N)
    x, w = _rand(M, K), _rand(N, K, scale=K**-0.5)
    r0 = _rand(M, N)
    g = (torch.rand(N, device=DEV) + 0.5).to(torch.bfloat16)
    ws = torch.zeros(16 << 20, device=DEV, dtype=torch.float32)
    r_f = r0.clone()
    xn = ops.linear_add_rmsnorm(x, w, r_f, g, 1e-5, ws)
    if xn is None:
        assert (M, N, K) != (64, 4096, 4096), "the Llama o_proj shape at 64 rows must take the fused path"
        pytest.skip("shape not on a split-K route")
    y = ops.linear(x, w, workspace=ws)
    r_u = r0.clone()
    xn_u = ops.rmsnorm(y, g, residual=r_u, residual_out=r_u, eps=1e-5)
    torch.cuda.synchronize()
    assert torch.equal(r_f, r_u)
    assert torch.equal(xn, xn_u)
    ref = (r0.float() + x.float() @ w.float().T)
    ref = ref * torch.rsqrt(ref.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    assert ((xn.float() - ref).abs().max() / ref.abs().max()).item() < 2e-2


def test_narrow_rows_not_taken():
    from mlmicroservicetemplate_amd import ops

    ws = torch.zeros(1 << 20, device=DEV, dtype=torch.float32)
    r = _rand(64, 1024)
    assert ops.linear_add_rmsnorm(_rand(64, 1024), _rand(1024, 1024), r, torch.ones(1024, device=DEV,
                                  dtype=torch.bfloat16), 1e-5, ws) is None


def test_llama_forward_fused_equals_unfused():
    from mlmicroservicetemplate_amd.models.llama import LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config(layers=3, hidden=2048, heads=16, kv_heads=4, head_dim=128, intermediate=4096)
    p = init_llama_shard(cfg, 1, 0, seed=7, device=DEV)
    outs = []
    for fused in (True, False):
        m = LlamaTP(p, cfg, backend="fused", device=DEV, max_batch=40, max_seq=256)
        m.fuse_add_norm = fused
        torch.manual_seed(4)
        B, S = 40, 3
        ids = torch.randint(3, cfg.vocab - 1, (B, S), device=DEV, dtype=torch.int32)
        lens = torch.full((B,), S, device=DEV, dtype=torch.int32)
        pos = torch.arange(S, device=DEV, dtype=torch.int32).unsqueeze(0).expand(B, S).contiguous()
        v, i = m.step(ids, pos, lens, decode=False, k=4)
        tok = i[:, 0].view(B, 1)
        v2, i2 = m.step(tok, lens.view(B, 1), lens + 1, decode=True, k=4)
        torch.cuda.synchronize()
        outs.append((v, i, v2, i2, getattr(m, "add_norm_fused", 0)))
        del m
    (fv, fi, fv2, fi2, nf), (uv, ui, uv2, ui2, nu) = outs
    assert nf > 0 and nu == 0
    assert torch.equal(fv, uv) and torch.equal(fi, ui)
    assert torch.equal(fv2, uv2) and torch.equal(fi2, ui2)
