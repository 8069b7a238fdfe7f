"""The 8-phase 256 x 256 tile GEMM (cfg 23, csrc/gemm_tile.hip gemm_8p_kernel): the same wave tile,
MFMA order per output element and epilogues as cfg 15, so every result must be BIT-identical to
cfg 15's, and close to an fp32 reference -- over ragged M / N, K-step counts 1..48 (the DMA schedule's
tail cases), several tiles per persistent block, the residual / GELU / SiLU-mul epilogues and the
LayerNorm-folding forms."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _ab(M, N, K, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    a = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) / K**0.5).to(torch.bfloat16)
    b = 0.1 * torch.randn(N, device=DEV, generator=g)
    r = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    return a, w, b, r


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 512, 128), (777, 2304, 192), (4096, 768, 3072),
                                   (16384, 2304, 768), (1000, 3072, 768), (513, 272, 256)])
@pytest.mark.parametrize("epi", ["bias", "gelu", "residual"])
def test_8phase_matches_cfg15_bitwise(M, N, K, epi):
    from mlmicroservicetemplate_amd import ops

    a, w, b, r = _ab(M, N, K, M + N + K)
    kw = {"act": ops.ACT_GELU} if epi == "gelu" else ({"residual": r} if epi == "residual" else {})
    ref15 = ops.gemm_tile(a, w, b, cfg=15, **kw)
    out = ops.gemm_tile(a, w, b, cfg=23, **kw)
    again = ops.gemm_tile(a, w, b, cfg=23, **kw)
    torch.cuda.synchronize()
    assert torch.equal(out, again)
    assert torch.equal(out, ref15), (out.float() - ref15.float()).abs().max().item()
    ref = a.float() @ w.float().T + b
    if epi == "gelu":
        ref = torch.nn.functional.gelu(ref)
    if epi == "residual":
        ref = ref + r.float()
    assert rel(out, ref) < 2e-2


def test_8phase_silu_mul_and_grid_cap():
    """SiLU-mul epilogue, and a capped grid (many tiles per persistent block)."""
    from mlmicroservicetemplate_amd import ops

    a, w, b, _ = _ab(2048, 1024, 512, 7)
    for cap in (0, 3, 17):
        ref15 = ops.gemm_tile(a, w, b, act=ops.ACT_SILU_MUL, cfg=15, grid_cap=cap)
        out = ops.gemm_tile(a, w, b, act=ops.ACT_SILU_MUL, cfg=23, grid_cap=cap)
        assert torch.equal(out, ref15)


@pytest.mark.parametrize("M", [4096, 777])
def test_8phase_layernorm_folding_forms(M):
    """gemm_tile_ln on cfg 23 (folded A, LN-residual + output-row partials through the re-aligned
    PART epilogue) == cfg 15 bitwise."""
    from mlmicroservicetemplate_amd import ops

    K, N = 768, 2304
    a, w, b, _ = _ab(M, N, K, 11)
    part = ops.ln_partials(M, K, a.device)
    h = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    tf = h.float().view(M, K // 128, 128)
    part.copy_(torch.stack([tf.sum(2), (tf * tf).sum(2)], 2).reshape(-1))
    c = w.float().sum(1).contiguous()
    o15 = ops.gemm_tile_ln(h, w, b, act=ops.ACT_GELU, fold_c=c, ln_part=part, cfg=15)
    o23 = ops.gemm_tile_ln(h, w, b, act=ops.ACT_GELU, fold_c=c, ln_part=part, cfg=23)
    assert torch.equal(o15, o23)
    # residual-LN + stats (N = 768 = the LN'd width)
    a2, w2, b2, _ = _ab(M, 768, 3072, 12)
    g = (1 + 0.1 * torch.randn(768, device=DEV)).contiguous()
    outs = []
    for cfg in (15, 23):
        sp = ops.ln_partials(M, 768, a.device)
        o = ops.gemm_tile_ln(a2, w2, b2, residual=h, ln_part=part, ln_g=g, stats_part=sp, cfg=cfg)
        outs.append((o, sp))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
