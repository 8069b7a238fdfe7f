"""Numerics of the hand-written HIP kernels vs plain-PyTorch fp32 references (SURVEY.md §4,
"Kernels (GPU)" row): exact ResNet-50 shapes (at small batch), every tile config, split-K,
residual/activation epilogues, padding/tails."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from mlmicroservicetemplate_amd import ops

    ops.lib()  # must load (fail loudly; no eager fallback)
    yield


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _conv_ref(x_nhwc, w_oihw, bias, stride, pad, act, res=None):
    y = F.conv2d(x_nhwc.permute(0, 3, 1, 2).float(), w_oihw.float(), stride=stride, padding=pad)
    y = y + bias.view(1, -1, 1, 1)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    if act == 1:
        y = torch.relu(y)
    return y


RESNET_CONV_SHAPES = [
    # cin, cout, k, s, p, h
    (64, 64, 1, 1, 0, 56),
    (64, 64, 3, 1, 1, 56),
    (64, 256, 1, 1, 0, 56),
    (256, 64, 1, 1, 0, 56),
    (256, 128, 1, 1, 0, 56),
    (128, 128, 3, 2, 1, 56),
    (256, 512, 1, 2, 0, 56),
    (512, 128, 1, 1, 0, 28),
    (128, 128, 3, 1, 1, 28),
    (256, 256, 3, 2, 1, 28),
    (512, 1024, 1, 2, 0, 28),
    (1024, 256, 1, 1, 0, 14),
    (256, 256, 3, 1, 1, 14),
    (512, 512, 3, 2, 1, 14),
    (1024, 2048, 1, 2, 0, 14),
    (2048, 512, 1, 1, 0, 7),
    (512, 512, 3, 1, 1, 7),
    (512, 2048, 1, 1, 0, 7),
]


@pytest.mark.parametrize("shape", RESNET_CONV_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_resnet_shapes(shape):
    from mlmicroservicetemplate_amd import ops

    cin, cout, k, s, p, h = shape
    torch.manual_seed(0)
    B = 2
    x = torch.randn(B, h, h, cin, device=DEV).to(torch.bfloat16)
    w = (torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(cout, device=DEV)
    ho = (h + 2 * p - k) // s + 1
    res = torch.randn(B, ho, ho, cout, device=DEV).to(torch.bfloat16)
    ref = _conv_ref(x, w, bias, s, p, 1, res)
    ws = torch.empty(64 << 20, device=DEV, dtype=torch.float32)
    for cfg in list(range(0, 32)):
        out = ops.conv2d_nhwc(x, ops.pack_conv_weight(w), bias, kernel=k, stride=s, pad=p, residual=res, act=1,
                              workspace=ws, cfg=cfg)
        torch.cuda.synchronize()
        assert rel_err(out, ref) < 2e-2, f"cfg {cfg}"
    # split-K
    out = ops.conv2d_nhwc(x, ops.pack_conv_weight(w), bias, kernel=k, stride=s, pad=p, residual=res, act=1,
                          workspace=ws, cfg=4, splitk=4)
    assert rel_err(out, ref) < 2e-2, "splitk"


def test_conv_stem():
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(1)
    B, h = 2, 224
    x3 = torch.randn(B, h, h, 3, device=DEV)
    x4 = torch.cat([x3, torch.zeros(B, h, h, 1, device=DEV)], dim=-1)
    x4p = torch.nn.functional.pad(x4, (0, 0, 3, 3, 3, 3)).to(torch.bfloat16)  # pre-padded image
    w = (torch.randn(64, 3, 7, 7, device=DEV) / 12.0).to(torch.bfloat16)
    bias = torch.randn(64, device=DEV)
    ref = _conv_ref(x4.to(torch.bfloat16)[..., :3], w, bias, 2, 3, 1)
    for cfg in list(range(0, 32)):
        out = ops.conv2d_nhwc(x4p, ops.pack_conv_weight(w), bias, kernel=7, stride=2, pad=0, act=1, cfg=cfg)
        assert out.shape == (B, 112, 112, 64)
        assert rel_err(out, ref) < 2e-2, f"cfg {cfg}"


@pytest.mark.parametrize("mnk", [(32, 1000, 2048), (1, 64, 64), (77, 136, 200), (300, 2304, 768), (513, 768, 3072)])
@pytest.mark.parametrize("act", [0, 1, 2, 3, 4])
def test_gemm(mnk, act):
    from mlmicroservicetemplate_amd import ops

    M, N, K = mnk
    torch.manual_seed(2)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K**0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    scale = torch.rand(N, device=DEV) + 0.5
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    y = (a.float() @ w.float().T) * scale + bias + res.float()
    ref = {0: y, 1: torch.relu(y), 2: F.gelu(y), 3: torch.tanh(y), 4: F.silu(y)}[act]
    ws = torch.empty(16 << 20, device=DEV, dtype=torch.float32)
    for cfg, sk in ((0, 0), (1, 1), (4, 2), (2, 3), (5, 1), (6, 2), (7, 1), (8, 3), (13, 1), (14, 2), (15, 1),
                    (16, 3), (17, 1), (18, 2), (19, 1), (20, 1), (21, 1), (22, 1), (23, 2), (24, 1), (25, 3),
                    (26, 1), (27, 2), (28, 1), (29, 1), (30, 1), (31, 2)):
        out = ops.gemm(a, w, bias, scale=scale, residual=res, act=act, workspace=ws, cfg=cfg, splitk=sk)
        assert rel_err(out, ref) < 2e-2, f"cfg {cfg} sk {sk}"


def test_gemm_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C-write (guide §3)."""
    from mlmicroservicetemplate_amd import ops

    n = 128
    eye = torch.eye(n, device=DEV).to(torch.bfloat16)
    b = torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n).remainder(97).to(torch.bfloat16)
    out = ops.gemm(eye, b)  # = I @ b.T
    assert torch.equal(out.float(), b.float().T)


def test_normalize_pool_head():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import IMAGENET_MEAN, IMAGENET_STD

    torch.manual_seed(3)
    img = torch.randint(0, 256, (3, 224, 224, 3), dtype=torch.uint8, device=DEV)
    out = ops.normalize_u8(img, IMAGENET_MEAN, IMAGENET_STD, pad=3)
    ref = (img.float() - torch.tensor(IMAGENET_MEAN, device=DEV)) / torch.tensor(IMAGENET_STD, device=DEV)
    assert out.shape == (3, 230, 230, 4)
    assert rel_err(out[:, 3:-3, 3:-3, :3], ref) < 1e-2
    assert out[..., 3].abs().max().item() == 0
    assert out[:, :3].abs().max().item() == 0 and out[:, :, -3:].abs().max().item() == 0

    x = torch.randn(2, 112, 112, 64, device=DEV).to(torch.bfloat16)
    mp = ops.maxpool2d_nhwc(x, 3, 2, 1)
    mref = F.max_pool2d(x.permute(0, 3, 1, 2).float(), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(mp.float(), mref)

    x = torch.randn(4, 7, 7, 2048, device=DEV).to(torch.bfloat16)
    ap = ops.avgpool_global_nhwc(x)
    assert rel_err(ap, x.float().mean(dim=(1, 2))) < 1e-2

    logits = torch.randn(32, 1000, device=DEV).to(torch.bfloat16)
    vals, idx = ops.softmax_topk(logits, 5)
    p = torch.softmax(logits.float(), -1)
    rv, ri = torch.topk(p, 5, dim=-1)
    assert torch.allclose(vals, rv, rtol=1e-3, atol=1e-5)
    # bf16 logits have ties; the selected ids must carry the top-k probabilities
    assert torch.allclose(p.gather(1, idx.long()), rv, rtol=1e-3, atol=1e-6)
    v2, i2 = ops.softmax_topk(logits.float(), 3, softmax=False)
    rv2, ri2 = torch.topk(logits.float(), 3, dim=-1)
    assert torch.allclose(v2, rv2) and torch.allclose(logits.float().gather(1, i2.long()), rv2)

    x = torch.randn(2 * 12 * 128, 128, device=DEV).to(torch.bfloat16)
    mask = torch.zeros(2, 128, device=DEV)
    mask[1, 100:] = -1e9
    sm = ops.softmax_rows(x, mask, rows_per_mask=12 * 128, scale=0.125)
    sref = torch.softmax(x.float() * 0.125 + mask.repeat_interleave(12 * 128, 0), -1)
    assert rel_err(sm, sref) < 1e-2

    x = torch.randn(64, 56, 56, 64, device=DEV).to(torch.bfloat16)
    sc, bi = torch.rand(64, device=DEV), torch.randn(64, device=DEV)
    y = ops.bn_act(x, sc, bi, relu=True)
    assert rel_err(y, torch.relu(x.float() * sc + bi)) < 1e-2


def test_resnet50_fused_matches_reference():
    from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50, resnet50_reference

    params = init_resnet50(0)
    torch.manual_seed(4)
    imgs = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device=DEV)
    model = ResNet50Fused(params, DEV, max_batch=32)
    logits = model(imgs).float()
    ref = resnet50_reference({k: v.to(DEV) for k, v in params.items()}, imgs)
    assert rel_err(logits, ref) < 2e-2
    vals, idx = model.classify(imgs, 5)
    top2 = ref.float().topk(2, dim=-1).values
    sure = (top2[:, 0] - top2[:, 1]) / ref.abs().max() > 1e-2
    assert torch.equal(idx[:, 0].long()[sure], ref.argmax(-1)[sure])


@pytest.mark.parametrize("rows,N,k", [(32, 1000, 5), (5, 8, 3), (7, 512, 50), (3, 2048, 10), (9, 1032, 1)])
@pytest.mark.parametrize("softmax", [True, False])
def test_softmax_topk_register_path(rows, N, k, softmax):
    """The register-resident bf16 head kernel (N % 8 == 0, N <= 2048) vs torch.topk."""
    from mlmicroservicetemplate_amd import ops

    torch.manual_seed(N + k)
    logits = (torch.randn(rows, N, device=DEV) * 3).to(torch.bfloat16)
    vals, idx = ops.softmax_topk(logits, k, softmax=softmax)
    ref = torch.softmax(logits.float(), -1) if softmax else logits.float()
    rv, _ri = torch.topk(ref, k, dim=-1)
    assert torch.allclose(vals, rv, rtol=1e-3, atol=1e-6)
    assert torch.allclose(ref.gather(1, idx.long()), rv, rtol=1e-3, atol=1e-6)
    assert (idx >= 0).all() and (idx < N).all()
    for r in range(rows):  # no index repeats
        assert len(set(idx[r].tolist())) == k


@pytest.mark.parametrize("shape", [(2, 14, 14, 64, 28, 28, 32, 2, 128), (3, 7, 7, 128, 7, 7, 64, 1, 256),
                                   (2, 5, 5, 64, 9, 9, 24, 2, 64)])
@pytest.mark.parametrize("cfg,splitk", [(0, 0), (4, 1), (1, 1), (9, 2), (13, 1), (15, 2), (16, 1)])
def test_conv1x1_dual(shape, cfg, splitk):
    """conv3 + downsample fused along K vs the two convolutions summed in fp32."""
    from mlmicroservicetemplate_amd import ops

    B, Ho, Wo, C1, H2, W2, C2, s2, cout = shape
    torch.manual_seed(B + C1)
    y = torch.randn(B, Ho, Wo, C1, device=DEV).to(torch.bfloat16)
    x = torch.randn(B, H2, W2, C2, device=DEV).to(torch.bfloat16)
    w1 = (torch.randn(cout, C1, device=DEV) / C1**0.5).to(torch.bfloat16)
    w2 = (torch.randn(cout, C2, device=DEV) / C2**0.5).to(torch.bfloat16)
    b = torch.randn(cout, device=DEV)
    ws = torch.empty(8 << 20, device=DEV, dtype=torch.float32)
    out = ops.conv1x1_dual(y, x, torch.cat([w1, w2], 1).contiguous(), b, stride2=s2, act="relu", workspace=ws,
                           cfg=cfg, splitk=splitk)
    xs = x[:, ::s2, ::s2, :][:, :Ho, :Wo, :]
    ref = torch.relu(y.float() @ w1.float().T + xs.float() @ w2.float().T + b)
    assert out.shape == (B, Ho, Wo, cout)
    assert rel_err(out, ref) < 2e-2


@pytest.mark.parametrize("B", [1, 3])
def test_stem_pool_fused_matches_three_kernels(B):
    """csrc/stem_pool.hip (normalise + 7x7/2 stem + ReLU + 3x3/2 max pool in one kernel) against the
    three-kernel path it replaces, and against the fp32 PyTorch reference of the same ops."""
    import torch.nn.functional as F

    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import IMAGENET_MEAN, IMAGENET_STD

    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(B)
    imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=g).to(dev)
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.05).to(dev)
    bias = (torch.randn(64, generator=g) * 0.5).to(dev)
    wp = ops.pack_conv_weight(w.to(torch.bfloat16))
    fused = ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD)
    x = ops.normalize_u8(imgs, IMAGENET_MEAN, IMAGENET_STD, pad=3)
    y = ops.conv2d_nhwc(x, wp, bias, kernel=7, stride=2, pad=0, act=ops.ACT_RELU,
                        workspace=torch.empty(1 << 20, device=dev, dtype=torch.float32))
    three = ops.maxpool2d_nhwc(y, 3, 2, 1)
    torch.cuda.synchronize()
    assert fused.shape == three.shape == (B, 56, 56, 64)
    diff = (fused.float() - three.float()).abs()
    assert diff.max().item() <= 0.02 * three.float().abs().max().item()  # fp32 summation order only
    assert (diff > 0).float().mean().item() < 0.02
    # fp32 reference
    mean = torch.tensor(IMAGENET_MEAN, device=dev).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=dev).view(1, 3, 1, 1)
    xr = ((imgs.permute(0, 3, 1, 2).float() - mean) / std).to(torch.bfloat16).float()
    ref = F.max_pool2d(F.relu(F.conv2d(xr, w.to(torch.bfloat16).float(), bias, stride=2, padding=3)), 3, 2, 1)
    ref = ref.permute(0, 2, 3, 1)
    err = ((fused.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("B", [1, 3, 32])
def test_stem_pool_v3_pipelined_matches_v2_and_fp32(B):
    """The software-pipelined stem tile loop (v3: double-buffered patch / stem tile, pool of tile
    t-1 inside tile t's MFMAs, bias as the MFMA's C, FMA normalisation) against the phase-serial v2
    loop -- every image row strip and both column halves, image borders included -- and against
    the fp32 PyTorch reference.  v3 adds the bias first and normalises with one FMA, so a few
    values round differently (one bf16 ulp)."""
    import torch.nn.functional as F

    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import IMAGENET_MEAN, IMAGENET_STD

    g = torch.Generator(device="cpu").manual_seed(20 + B)
    imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=g).to(DEV)
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    wp = ops.pack_conv_weight(w)
    bias = (torch.randn(64, generator=g) * 0.5).to(DEV)
    lib = ops.lib()
    old = lib.mls_stem_set_version(2)
    try:
        v2 = ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD)
        lib.mls_stem_set_version(3)
        v3 = ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD)
        torch.cuda.synchronize()
    finally:
        lib.mls_stem_set_version(old)
    assert v3.shape == (B, 56, 56, 64)
    diff = (v3.float() - v2.float()).abs()
    assert diff.max().item() <= 0.02 * v2.float().abs().max().item()
    assert (diff > 0).float().mean().item() < 0.05
    # zero-forced border rows / columns and every tile position agree on which outputs are zero
    assert torch.equal(v3 == 0, v2 == 0) or ((v3 == 0) != (v2 == 0)).float().mean().item() < 1e-3
    mean = torch.tensor(IMAGENET_MEAN, device=DEV).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=DEV).view(1, 3, 1, 1)
    xr = ((imgs.permute(0, 3, 1, 2).float() - mean) / std).to(torch.bfloat16).float()
    ref = F.max_pool2d(F.relu(F.conv2d(xr, w.float(), bias, stride=2, padding=3)), 3, 2, 1).permute(0, 2, 3, 1)
    err = ((v3.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("B", [1, 3])
def test_stem_pool_conv1_fused(B):
    """The stem kernel with layer1.0's 1x1 conv on its pooled tiles: pooled map unchanged, t1 equal
    to the separate conv kernel on that map (and to fp32 within bf16 rounding)."""
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import IMAGENET_MEAN, IMAGENET_STD

    g = torch.Generator(device="cpu").manual_seed(10 + B)
    imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, generator=g).to(DEV)
    wp = ops.pack_conv_weight((torch.randn(64, 3, 7, 7, generator=g) * 0.05).to(torch.bfloat16).to(DEV))
    bias = (torch.randn(64, generator=g) * 0.5).to(DEV)
    w1 = (torch.randn(64, 64, generator=g) / 8).to(torch.bfloat16).to(DEV)
    b1 = (torch.randn(64, generator=g) * 0.1).to(DEV)
    lib = ops.lib()
    old = lib.mls_stem_set_version(2)  # the phase-serial loop: the same arithmetic as the conv1 kernel
    try:
        pooled = ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD)
    finally:
        lib.mls_stem_set_version(old)
    x, t1 = ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD, conv1_w=w1, conv1_b=b1)
    assert torch.equal(x, pooled)
    # the default (pipelined v3) loop rounds a few values differently (bias first, FMA normalisation)
    assert rel_err(ops.stem_pool_u8(imgs, wp, bias, IMAGENET_MEAN, IMAGENET_STD), pooled) < 1e-2
    sep = ops.conv2d_nhwc(x, w1.view(64, 1, 1, 64), b1, kernel=1, act=ops.ACT_RELU)
    assert rel_err(t1, sep) < 1e-2
    ref = torch.relu(x.float() @ w1.float().T + b1)
    assert rel_err(t1, ref) < 1e-2


@pytest.mark.parametrize("B,H,W,cin,cout,resid", [
    (2, 56, 56, 64, 64, False),   # layer1 conv2: 4 rows x 56 per tile
    (2, 28, 28, 128, 128, False),  # layer2: 7 x 28
    (2, 14, 14, 256, 256, False),  # layer3: whole image
    (8, 7, 7, 512, 512, False),    # layer4: 4 images per tile
    (3, 10, 12, 32, 64, True),     # odd geometry + residual epilogue
])
def test_conv3x3_halo_matches_reference(B, H, W, cin, cout, resid):
    """csrc/conv3x3_halo.hip (halo-tiled direct 3x3 / s1 / p1) vs the fp32 PyTorch conv, and vs the
    implicit-GEMM kernel it can replace."""
    from mlmicroservicetemplate_amd import ops

    g = torch.Generator(device="cpu").manual_seed(H * cin + B)
    x = torch.randn(B, H, W, cin, generator=g).to(DEV).to(torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(DEV).to(torch.bfloat16)
    bias = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    res = torch.randn(B, H, W, cout, generator=g).to(DEV).to(torch.bfloat16) if resid else None
    assert ops.conv3x3_halo_geometry(B, H, W) is not None
    assert ops.conv3x3_halo_geometry(B, H, W, variant=2) is not None
    ref = _conv_ref(x, w, bias, 1, 1, 1, res)
    ws = torch.empty(4 * B * H * W * cout, device=DEV, dtype=torch.float32)
    for variant, sk in ((1, 1), (0, 1), (0, 2), (0, 4), (2, 1), (2, 2), (2, 4)):
        if (cin // 32) % sk:
            continue
        for _ in range(2):  # the second launch checks the split-K counters were left at zero
            out = ops.conv3x3_halo(x, ops.pack_conv_weight(w), bias, act=ops.ACT_RELU, residual=res,
                                   variant=variant, splitk=sk, workspace=ws)
            assert rel_err(out, ref) < 2e-2, (variant, sk)
    if cin % 64:
        return  # the implicit-GEMM kernel needs Cin % 64 == 0
    gemm = ops.conv2d_nhwc(x, ops.pack_conv_weight(w), bias, kernel=3, stride=1, pad=1, act=ops.ACT_RELU,
                           residual=res, workspace=torch.empty(8 << 20, device=DEV, dtype=torch.float32))
    assert rel_err(out, gemm) < 2e-2


@pytest.mark.parametrize("M,N,K,act", [(32, 28672, 4096, "silu_mul"), (32, 4096, 4096, "none"),
                                       (64, 4096, 14336, "none"), (64, 28672, 4096, "silu_mul"),
                                       (128, 4096, 4096, "none"), (128, 4096, 14336, "none")])
def test_linear_gemm_plan_shapes(M, N, K, act):
    """ops.linear on the shapes tuned/gemm_plan_gfx950.json routes to a fixed native cfg / split-K."""
    from mlmicroservicetemplate_amd import ops

    assert (M, N, K) in ops.gemm_plan()
    g = torch.Generator(device="cpu").manual_seed(M + N)
    a = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K**0.5).to(DEV, torch.bfloat16)
    res = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16) if act == "none" else None
    ws = torch.empty(32 << 20, device=DEV)
    y = ops.linear(a, w, act=act, residual=res, workspace=ws)
    ref = a.float() @ w.float().t()
    if act == "silu_mul":
        r = ref.view(M, N // 16, 2, 8)
        ref = (F.silu(r[:, :, 0]) * r[:, :, 1]).reshape(M, N // 2)
    else:
        ref = ref + res.float()
    assert rel_err(y, ref) < 2e-2
