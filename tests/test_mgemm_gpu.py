"""csrc/mgemm.hip medium-M weight-streaming GEMM (ops.mgemm, 17..256-row decode batches) vs a plain
PyTorch fp32 reference: row-tile variants (M <= 64 / 128 / 256), split-K 1..8, bias, residual,
SiLU-mul, a strided A, and bit-identical repeat launches."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,split", [(17, 64, 256, 1), (64, 128, 512, 2), (65, 192, 1024, 4), (128, 256, 2048, 8),
                                         (200, 512, 1024, 1), (256, 1024, 4096, 0), (256, 4096, 4096, 4),
                                         (129, 320, 1792, 7), (31, 64, 14336, 0)])
def test_mgemm_plain_bias_residual(M, N, K, split):
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(M + N + K)
    x, w = _rand(M, K), _rand(N, K, scale=K**-0.5)
    b, res = torch.randn(N, device=DEV) * 0.1, _rand(M, N)
    out = ops.mgemm(x, w, b, residual=res, splitk=split)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().T + b + res.float()
    assert out.shape == (M, N)
    assert rel_err(out, ref) < 1e-2
    out2 = ops.mgemm(x, w, b, residual=res, splitk=split)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("M,split", [(48, 1), (100, 2), (256, 4)])
def test_mgemm_silu_mul(M, split):
    from mlmicroservicetemplate_amd import ops

    K, N = 1024, 512
    torch.manual_seed(M)
    x, w = _rand(M, K), _rand(N, K, scale=K**-0.5)
    b = torch.randn(N, device=DEV) * 0.1
    out = ops.mgemm(x, w, b, act="silu_mul", splitk=split)
    y = x.float() @ w.float().T + b
    g = y.view(M, N // 16, 2, 8)
    ref = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(M, N // 2)
    assert out.shape == (M, N // 2)
    assert rel_err(out, ref) < 1e-2


def test_mgemm_strided_a_and_no_bias():
    """A as a column slice of a wider buffer (row stride > K), no bias / residual."""
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(3)
    M, N, K = 96, 256, 512
    big = _rand(M, K + 64)
    x = big[:, 32:32 + K]
    w = _rand(N, K, scale=K**-0.5)
    out = ops.mgemm(x, w, splitk=2)
    ref = x.float() @ w.float().T
    assert rel_err(out, ref) < 1e-2


def test_mgemm_rejects_bad_shapes():
    from mlmicroservicetemplate_amd import ops

    with pytest.raises(ValueError):
        ops.mgemm(_rand(300, 256), _rand(64, 256))
    with pytest.raises(ValueError):
        ops.mgemm(_rand(32, 256), _rand(48, 256))
    with pytest.raises(ValueError):
        ops.mgemm(_rand(32, 200), _rand(64, 200))
