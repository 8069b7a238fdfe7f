"""csrc/skinny_gemm.hip packed-weight decode GEMM (mls_skinny_packed / mls_skinny_pack) vs a plain
PyTorch fp32 reference, every launch variant (cache policy x waves x granules per trip)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def test_pack_matches_reference_layout():
    from mlmicroservicetemplate_amd import ops

    w = _rand(96, 320)
    assert torch.equal(ops.pack_skinny(w), ops.pack_skinny_reference(w))


@pytest.mark.parametrize("variant", list(range(14)) + [17, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("M,N,K", [(1, 256, 4096), (3, 128, 1024), (2, 64, 14336), (4, 64, 8192), (2, 48, 96),
                                   (8, 128, 4096), (16, 64, 1024), (5, 32, 14336), (24, 96, 2048), (32, 6144, 256)])
def test_packed_plain(variant, M, N, K):
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(variant + M + N)
    x, w = _rand(M, K), _rand(N, K, scale=K**-0.5)
    b, res = torch.randn(N, device=DEV) * 0.1, _rand(M, N)
    out = ops.skinny_packed(x, ops.pack_skinny(w), N, bias=b, residual=res, variant=variant)
    ref = x.float() @ w.float().T + b + res.float()
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize("variant", [0, 3, 5, 6, 9, 25, 17, 11, 12, 13])
@pytest.mark.parametrize("M", [1, 4, 8, 16, 17, 32])
def test_packed_add_norm_silu_mul(variant, M):
    """The decode gate_up form: RMSNorm(x + delta) with the gain folded into W, SiLU-mul epilogue,
    x + delta written back to the residual stream."""
    from mlmicroservicetemplate_amd import ops

    K, N = 512, 256
    torch.manual_seed(10 * variant + M)
    x, d = _rand(M, K), _rand(M, K)
    gain = torch.rand(K, device=DEV) + 0.5
    w = ops.interleave_gate_up(_rand(N // 2, K, scale=K**-0.5), _rand(N // 2, K, scale=K**-0.5))
    r_out = torch.empty_like(x)
    out = ops.skinny_packed(x, ops.pack_skinny(ops.fold_norm(w, gain)), N, delta=d, resid_out=r_out, norm=True,
                            act="silu_mul", variant=variant)
    h = (x.float() + d.float()).to(torch.bfloat16)
    assert torch.equal(r_out, h)
    hf = h.float()
    xn = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * gain
    y = xn @ w.float().T
    g, u = y.view(M, N // 16, 2, 8)[:, :, 0].reshape(M, -1), y.view(M, N // 16, 2, 8)[:, :, 1].reshape(M, -1)
    ref = torch.nn.functional.silu(g) * u
    assert rel_err(out, ref) < 2e-2


def test_packed_matches_row_major_skinny():
    """Same products as the row-major skinny kernel (fused-norm QKV shape at batch 1)."""
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(3)
    K, N = 4096, 768
    x, w = _rand(1, K), _rand(N, K, scale=K**-0.5)
    a = ops.gemm_rmsnorm(x, w)
    b = ops.skinny_packed(x, ops.pack_skinny(w), N, norm=True)
    assert rel_err(b, a) < 1e-2


def test_packed_rejects_bad_shapes():
    from mlmicroservicetemplate_amd import ops

    w = _rand(64, 256)
    wp = ops.pack_skinny(w)
    with pytest.raises(ValueError):
        ops.skinny_packed(_rand(33, 256), wp, 64)  # M > 32
    with pytest.raises(ValueError):
        ops.skinny_packed(_rand(1, 256), wp, 48)  # wp size mismatch
    with pytest.raises(ValueError):
        ops.pack_skinny(_rand(64, 200))  # K % 32


@pytest.mark.parametrize("lens_list", [[300], [1, 64, 65, 700], [129, 20]])
def test_packed_combine_matches_attention_then_gemm(lens_list):
    """o-projection with the split-KV combine in its prologue == decode attention (own combine
    launch) followed by the packed GEMM; rows that fit one split come from the direct-written A."""
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(len(lens_list))
    B, Hq, Hkv, D, L = len(lens_list), 32, 8, 128, 1024
    kc = torch.randn(B, L, Hkv, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor(lens_list, device=DEV, dtype=torch.int32)
    N = 4096
    w = _rand(N, Hq * D, scale=(Hq * D) ** -0.5)
    wp = ops.pack_skinny(w)
    res = _rand(B, N)
    a_ref = ops.decode_attention(q, kc, vc, lens, Hq, Hkv, D, max_len=L)
    want = ops.skinny_packed(a_ref, wp, N, residual=res)
    a, parts = ops.decode_attention(q, kc, vc, lens, Hq, Hkv, D, max_len=L, combine=False)
    got = ops.skinny_packed_combine(a, parts, wp, N, residual=res)
    assert rel_err(got, want) < 1e-2


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(1, 256, 4096), (3, 128, 1024), (2, 64, 14336), (4, 48, 128)])
def test_fp8_plain_matches_emulation(variant, M, N, K):
    """W8A8 e4m3 kernel == an fp32 emulation of the same quantisation (and within fp8 error of
    the bf16 product)."""
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(variant * 7 + M)
    x, w = _rand(M, K), _rand(N, K, scale=K**-0.5)
    b, res = torch.randn(N, device=DEV) * 0.1, _rand(M, N)
    wq, sw = ops.pack_skinny_fp8(w)
    out = ops.skinny_fp8(x, wq, sw, N, bias=b, residual=res, variant=variant)
    emu = ops.fp8_reference(x, w) + b + res.float()
    assert rel_err(out, emu) < 1e-2
    exact = x.float() @ w.float().T + b + res.float()
    assert rel_err(out, exact) < 6e-2


def test_fp8_identity_asymmetric():
    """A = I rows against an asymmetric W catches a transposed operand map."""
    from mlmicroservicetemplate_amd import ops

    K, N = 64, 16
    w = (torch.arange(N * K, device=DEV, dtype=torch.float32).view(N, K).remainder(13) - 6).to(torch.bfloat16)
    for r in range(4):
        x = torch.zeros(1, K, device=DEV, dtype=torch.bfloat16)
        x[0, 5 + 9 * r] = 1.0
        wq, sw = ops.pack_skinny_fp8(w)
        out = ops.skinny_fp8(x, wq, sw, N)
        assert torch.allclose(out.float()[0], w.float()[:, 5 + 9 * r], atol=0.05 * 6), r


@pytest.mark.parametrize("M", [1, 4])
def test_fp8_add_norm_silu_mul(M):
    from mlmicroservicetemplate_amd import ops

    K, N = 1024, 256
    torch.manual_seed(M)
    x, d = _rand(M, K), _rand(M, K)
    gain = torch.rand(K, device=DEV) + 0.5
    w = ops.interleave_gate_up(_rand(N // 2, K, scale=K**-0.5), _rand(N // 2, K, scale=K**-0.5))
    wf = ops.fold_norm(w, gain)
    wq, sw = ops.pack_skinny_fp8(wf)
    r_out = torch.empty_like(x)
    out = ops.skinny_fp8(x, wq, sw, N, delta=d, resid_out=r_out, norm=True, act="silu_mul")
    h = (x.float() + d.float()).to(torch.bfloat16)
    assert torch.equal(r_out, h)
    rstd = torch.rsqrt(h.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    y = ops.fp8_reference(h, wf) * rstd
    g_, u_ = y.view(M, N // 16, 2, 8)[:, :, 0].reshape(M, -1), y.view(M, N // 16, 2, 8)[:, :, 1].reshape(M, -1)
    ref = torch.nn.functional.silu(g_) * u_
    assert rel_err(out, ref) < 2e-2
