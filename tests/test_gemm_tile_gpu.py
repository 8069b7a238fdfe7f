"""ops.gemm_tile (csrc/gemm_tile.hip) per tile variant against a plain fp32 PyTorch reference of the
same op: ragged M / N (rows and columns past the edge are range-checked, never stored), every
epilogue (bias, GELU, residual, SiLU-mul pairing) and persistent blocks that walk several tiles
each (grid_cap) so the DMA ring runs across tile boundaries."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def _cfgs():
    from mlmicroservicetemplate_amd import ops

    return sorted(c for c in ops.GEMM_TILE_CFGS if c != 8)  # 8: ping-pong reference variant, spills


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 12, 15, 16, 21, 22])
@pytest.mark.parametrize("M,N,K,cap", [(300, 528, 192, 0), (1024, 1280, 512, 3), (4096, 768, 768, 0)])
def test_gemm_tile_epilogues(cfg, M, N, K, cap):
    from mlmicroservicetemplate_amd import ops

    assert cfg in _cfgs()
    torch.manual_seed(cfg * 7 + M)
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=DEV) * 2 - 1) / K**0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV) * 0.1
    r = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    y = a.float() @ w.float().T + b
    out = ops.gemm_tile(a, w, b, cfg=cfg, grid_cap=cap)
    assert rel(out, y) < 1e-2
    out = ops.gemm_tile(a, w, b, act=ops.ACT_GELU, cfg=cfg, grid_cap=cap)
    assert rel(out, torch.nn.functional.gelu(y)) < 1e-2
    out = ops.gemm_tile(a, w, None, residual=r, cfg=cfg, grid_cap=cap)
    assert rel(out, y - b + r.float()) < 1e-2
    # columns past N are never written: a wider output view keeps its sentinel
    wide = torch.full((M, N + 16), 7.0, device=DEV, dtype=torch.bfloat16)
    ops.lib().mls_gemm_tile(a.data_ptr(), w.data_ptr(), b.data_ptr(), 0, wide.data_ptr(), M, N, K, ops.ACT_NONE,
                            N + 16, N, cfg, cap, 1, None, 0, None, 0, ops.stream_ptr(a.device))
    torch.cuda.synchronize()
    assert rel(wide[:, :N], y) < 1e-2 and bool((wide[:, N:] == 7.0).all())
    g = (w[: N // 2] if (N // 2) % 16 == 0 else w[:N // 2 // 16 * 16]).contiguous()
    u = w[N - g.shape[0]:].contiguous()
    gu = ops.interleave_gate_up(g, u)
    out = ops.gemm_tile(a, gu, None, act=ops.ACT_SILU_MUL, cfg=cfg, grid_cap=cap)
    ref = torch.nn.functional.silu(a.float() @ g.float().T) * (a.float() @ u.float().T)
    assert out.shape == ref.shape and rel(out, ref) < 1e-2


@pytest.mark.parametrize("cfg", [1, 2, 15, 16])
@pytest.mark.parametrize("M,N,K,S", [(300, 528, 256, 2), (4096, 768, 3072, 3), (1024, 1280, 1536, 4)])
def test_gemm_tile_splitk(cfg, M, N, K, S):
    """In-launch split-K combine: every epilogue kind matches fp32 and the counters come back to
    zero (the next launch, and a graph replay, start clean); repeated launches agree bit for bit."""
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(cfg + S)
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=DEV) * 2 - 1) / K**0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV) * 0.1
    r = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    ws = torch.zeros(16 << 20, device=DEV, dtype=torch.float32)
    y = a.float() @ w.float().T + b
    o1 = ops.gemm_tile(a, w, b, cfg=cfg, splitk=S, workspace=ws)
    assert rel(o1, y) < 1e-2
    assert rel(ops.gemm_tile(a, w, b, act=ops.ACT_GELU, cfg=cfg, splitk=S, workspace=ws), torch.nn.functional.gelu(y)) < 1e-2
    assert rel(ops.gemm_tile(a, w, None, residual=r, cfg=cfg, splitk=S, workspace=ws), y - b + r.float()) < 1e-2
    gu = ops.interleave_gate_up(w[:256].contiguous(), w[256:512].contiguous())
    ref = torch.nn.functional.silu(a.float() @ w[:256].float().T) * (a.float() @ w[256:512].float().T)
    assert rel(ops.gemm_tile(a, gu, None, act=ops.ACT_SILU_MUL, cfg=cfg, splitk=S, workspace=ws), ref) < 1e-2
    torch.cuda.synchronize()
    assert int(ops.split_counters(ws).abs().sum().item()) == 0
    for _ in range(3):
        assert torch.equal(ops.gemm_tile(a, w, b, cfg=cfg, splitk=S, workspace=ws), o1)
    g = torch.cuda.CUDAGraph()
    out = torch.empty_like(o1)
    with torch.cuda.graph(g):
        ops.gemm_tile(a, w, b, cfg=cfg, splitk=S, workspace=ws, out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, o1)
