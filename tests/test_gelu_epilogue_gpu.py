"""The tile-GEMM epilogue GELU (common.h gelu_fast: the tanh form, or the erf form when the library
is built with MLS_GELU_ERF=1) against PyTorch's exact erf GELU over a dense grid of bf16 inputs.

The product is set up to be exact: w = I (bf16), so every output element is GELU(x) of one bf16
input x.  Bound: |out - gelu_erf(x)| <= 4.7e-4 (the tanh form's largest deviation, at x = 2.70)
plus half a bf16 ulp of the stored output."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_epilogue_gelu_vs_erf_gelu_dense_grid():
    from mlmicroservicetemplate_amd import ops

    K = N = 128
    M = 512  # the tile kernel's row range (>= TILE_MIN_M)
    xs = torch.linspace(-8.0, 8.0, M * K).to(torch.bfloat16)  # bf16-exact inputs
    a = xs.view(M, K).to(DEV)
    w = torch.eye(N, K, dtype=torch.bfloat16, device=DEV)
    out = ops.gemm_tile(a, w, None, act=ops.ACT_GELU).float()
    ref = torch.nn.functional.gelu(a.float(), approximate="none")
    err = (out - ref).abs()
    half_ulp = torch.where(ref.abs() > 0, torch.ldexp(torch.ones_like(ref), torch.frexp(ref.abs())[1] - 9),
                           torch.zeros_like(ref))
    worst = (err - half_ulp).max().item()
    assert worst <= 4.7e-4 + 1e-7, f"epilogue GELU off the erf GELU by {worst:.3e} beyond half a bf16 ulp"
    # where |GELU| is not tiny the two forms round to the same bf16 value almost everywhere (on the
    # negative tail, |GELU(x)| ~ 1e-3 .. 1e-8, the 4.7e-4 absolute difference spans many bf16 ulps)
    big = ref.abs() > 0.5
    exact = (out[big].to(torch.bfloat16) == ref[big].to(torch.bfloat16)).float().mean().item()
    assert exact > 0.9, f"only {exact:.3f} of the |GELU| > 0.5 outputs round to the erf GELU's bf16 value"
