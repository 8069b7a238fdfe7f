"""LayerNorm folding algebra (ops.fold_layernorm) on the CPU: rstd * (h @ W'.T - mu * c) + b' equals
LN(h) @ W.T + b -- the identity the tile kernel's EPI 4 epilogue evaluates."""
import torch

from mlmicroservicetemplate_amd import ops


def test_fold_layernorm_identity():
    g = torch.Generator().manual_seed(0)
    M, K, N = 64, 768, 256
    h = (torch.randn(M, K, generator=g) * 2 + 0.5).to(torch.bfloat16).float()
    w = (torch.randn(N, K, generator=g) / K**0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g)
    gam = 1 + 0.2 * torch.randn(K, generator=g)
    bet = 0.1 * torch.randn(K, generator=g)
    w2, c, b2 = ops.fold_layernorm(w, b, gam, bet)
    assert w2.dtype == torch.bfloat16 and c.dtype == torch.float32 and b2.dtype == torch.float32
    mu = h.mean(1, keepdim=True)
    rstd = torch.rsqrt(h.var(1, unbiased=False, keepdim=True) + 1e-12)
    folded = rstd * (h @ w2.float().T - mu * c[None, :]) + b2[None, :]
    ref = torch.nn.functional.layer_norm(h, (K,), gam, bet, 1e-12) @ w.float().T + b
    err = ((folded - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-2, err  # bf16 rounding of W' only
    # c is the sum of the bf16 W' actually multiplied, so a constant row folds to exactly the bias
    const = torch.full((1, K), 3.0)
    assert torch.allclose(const @ w2.float().T - 3.0 * c[None, :], torch.zeros(1, N), atol=1e-3)


def test_ln_foldable_shapes():
    assert ops.ln_foldable(4096, 2304, 768)
    assert ops.ln_foldable(16384, 768, 3072)
    assert not ops.ln_foldable(128, 768, 768)  # below TILE_MIN_M: the model keeps explicit LNs
    assert not ops.ln_foldable(4096, 770, 768)
    assert not ops.ln_foldable(4096, 768, 100)
    assert not ops.ln_foldable(4096, 704, 768)  # statistics come in 128-column blocks


def test_layernorm_from_partials_matches_torch():
    g = torch.Generator().manual_seed(1)
    M, W = 37, 768
    h = (torch.randn(M, W, generator=g) * 3 + 1).to(torch.bfloat16)
    part = torch.empty(M * (W // 128) * 2)
    hf = h.float().view(M, W // 128, 128)
    part.view(M, W // 128, 2)[:, :, 0] = hf.sum(2)
    part.view(M, W // 128, 2)[:, :, 1] = (hf * hf).sum(2)
    mu, rstd = ops.layernorm_from_partials(h, part)
    assert torch.allclose(mu, h.float().mean(1), atol=1e-5)
    assert torch.allclose(rstd, torch.rsqrt(h.float().var(1, unbiased=False) + 1e-12), rtol=1e-4)
