"""csrc/conv_chain.hip: a bottleneck's conv3 (+ residual / + downsample) chained with the next
block's conv1 in one kernel, vs a plain-PyTorch fp32 reference and vs the two separate conv
kernels it replaces (which it must match bit for bit on y: same rounding, same K order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from mlmicroservicetemplate_amd import ops

    ops.lib()
    yield


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


# (B, H, K, N1, N2): layer1 / layer2 boundaries at small batch, plus M tails (M % 128 != 0)
SHAPES = [(2, 56, 64, 256, 64), (2, 56, 64, 256, 128), (2, 28, 128, 512, 128), (3, 9, 64, 256, 64),
          (1, 7, 128, 512, 128), (2, 28, 128, 512, 256), (2, 14, 256, 1024, 256), (3, 7, 256, 1024, 256)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_chain_matches_reference_and_two_kernels(shape):
    from mlmicroservicetemplate_amd import ops

    B, H, K, N1, N2 = shape
    torch.manual_seed(sum(shape))
    t2 = torch.relu(_rand(B, H, H, K))
    res = _rand(B, H, H, N1)
    w3 = _rand(N1, K, scale=K**-0.5)
    w1 = _rand(N2, N1, scale=N1**-0.5)
    b3, b1 = torch.randn(N1, device=DEV) * 0.1, torch.randn(N2, device=DEV) * 0.1
    y, t1 = ops.conv1x1_chain(t2, w3, b3, w1, b1, residual=res)
    # fp32 reference (y rounded to bf16 as the network stores it)
    y_ref = torch.relu(t2.float() @ w3.float().T + b3 + res.float())
    t1_ref = torch.relu(y_ref.to(torch.bfloat16).float() @ w1.float().T + b1)
    assert rel_err(y, y_ref) < 1e-2 and rel_err(t1, t1_ref) < 2e-2
    # the unchained path: conv3 with the residual epilogue, then conv1
    y2 = ops.conv2d_nhwc(t2, w3.view(N1, 1, 1, K), b3, kernel=1, residual=res, act=ops.ACT_RELU)
    t12 = ops.conv2d_nhwc(y2, w1.view(N2, 1, 1, N1), b1, kernel=1, act=ops.ACT_RELU)
    assert torch.equal(y, y2)
    assert rel_err(t1, t12) < 1e-2


@pytest.mark.parametrize("stride2,H2", [(1, 56), (2, 17)])
def test_chain_dual_downsample(stride2, H2):
    """The stage-opening form: [t2 | x strided] . [W3 ; Wd]^T (no residual), then conv1."""
    from mlmicroservicetemplate_amd import ops

    B, Ka, Kb, N1, N2 = 2, 64, 64, 256, 64
    Ho = (H2 - 1) // stride2 + 1
    torch.manual_seed(stride2)
    t2 = torch.relu(_rand(B, Ho, Ho, Ka))
    x = _rand(B, H2, H2, Kb)
    w3 = _rand(N1, Ka, scale=Ka**-0.5)
    wd = _rand(N1, Kb, scale=Kb**-0.5)
    w1 = _rand(N2, N1, scale=N1**-0.5)
    b3, b1 = torch.randn(N1, device=DEV) * 0.1, torch.randn(N2, device=DEV) * 0.1
    wcat = torch.cat([w3, wd], 1).contiguous()
    y, t1 = ops.conv1x1_chain(t2, wcat, b3, w1, b1, a2=x, stride2=stride2)
    xs = x[:, ::stride2, ::stride2, :][:, :Ho, :Ho, :]
    y_ref = torch.relu(t2.float() @ w3.float().T + xs.float() @ wd.float().T + b3)
    t1_ref = torch.relu(y_ref.to(torch.bfloat16).float() @ w1.float().T + b1)
    assert rel_err(y, y_ref) < 1e-2 and rel_err(t1, t1_ref) < 2e-2
    y2 = ops.conv1x1_dual(t2, x, wcat, b3, stride2=stride2, act=ops.ACT_RELU)
    assert rel_err(y, y2) < 1e-2


@pytest.mark.parametrize("cw", [32, 64])
def test_chain_layer2_chunk_widths(cw):
    """Both instantiations of the layer2 boundary (64-wide stages, one block per CU; 32-wide,
    two per CU) compute the same y / t1."""
    from mlmicroservicetemplate_amd import ops

    B, H, K, N1, N2 = 2, 28, 128, 512, 128
    torch.manual_seed(cw)
    t2, res = torch.relu(_rand(B, H, H, K)), _rand(B, H, H, N1)
    w3, w1 = _rand(N1, K, scale=K**-0.5), _rand(N2, N1, scale=N1**-0.5)
    b3, b1 = torch.randn(N1, device=DEV) * 0.1, torch.randn(N2, device=DEV) * 0.1
    try:
        ops.set_chain_l2_cw(cw)
        y, t1 = ops.conv1x1_chain(t2, w3, b3, w1, b1, residual=res)
    finally:
        ops.set_chain_l2_cw(0)
    y_ref = torch.relu(t2.float() @ w3.float().T + b3 + res.float())
    t1_ref = torch.relu(y_ref.to(torch.bfloat16).float() @ w1.float().T + b1)
    assert rel_err(y, y_ref) < 1e-2 and rel_err(t1, t1_ref) < 2e-2


@pytest.mark.parametrize("n2", [128, 256])
def test_chain_layer2_row_tile_64(n2):
    """The 64-row tile of the layer2 boundaries (twice the blocks of the 128-row default; ragged
    last tile at B = 3) computes the same y / t1."""
    from mlmicroservicetemplate_amd import ops

    B, H, K, N1 = 3, 28, 128, 512
    torch.manual_seed(n2)
    t2, res = torch.relu(_rand(B, H, H, K)), _rand(B, H, H, N1)
    w3, w1 = _rand(N1, K, scale=K**-0.5), _rand(n2, N1, scale=N1**-0.5)
    b3, b1 = torch.randn(N1, device=DEV) * 0.1, torch.randn(n2, device=DEV) * 0.1
    try:
        ops.lib().mls_chain_set_l2_bm(64)
        y, t1 = ops.conv1x1_chain(t2, w3, b3, w1, b1, residual=res)
    finally:
        ops.lib().mls_chain_set_l2_bm(128)
    y_ref = torch.relu(t2.float() @ w3.float().T + b3 + res.float())
    t1_ref = torch.relu(y_ref.to(torch.bfloat16).float() @ w1.float().T + b1)
    assert rel_err(y, y_ref) < 1e-2 and rel_err(t1, t1_ref) < 2e-2


def test_chain_rejects_unsupported_shapes():
    from mlmicroservicetemplate_amd import ops

    t2 = _rand(1, 7, 7, 512)
    with pytest.raises(ValueError):  # a layer4 boundary: not instantiated
        ops.conv1x1_chain(t2, _rand(2048, 512), None, _rand(512, 2048), None, residual=_rand(1, 7, 7, 2048))


def test_resnet50_chain_matches_unchained():
    """The network with the layer1 / layer2 boundaries chained computes what the per-conv
    kernels compute (and stays within the fp32 reference's tolerance)."""
    from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50, resnet50_reference

    params = init_resnet50(0)
    torch.manual_seed(5)
    imgs = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device=DEV)
    model = ResNet50Fused(params, DEV, max_batch=32)
    assert model.chain
    chained = model(imgs).float()
    model.chain = False
    plain = model(imgs).float()
    assert rel_err(chained, plain) < 1e-2
    ref = resnet50_reference({k: v.to(DEV) for k, v in params.items()}, imgs)
    assert rel_err(chained, ref) < 5e-2
