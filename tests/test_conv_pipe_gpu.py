"""Pipelined halo-tiled 3x3 conv (csrc/conv3x3_pipe.hip) vs a plain PyTorch fp32 conv2d of the same
bf16 operands: every variant on the four ResNet-50 bottleneck conv2 shapes, with and without the
in-launch split-K reduction and several items per block, replayed twice (the split-K arrival
counters reset themselves), plus small / odd batches."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _ref(x, w_oihw, b, relu=True):
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w_oihw.float(), padding=1) + b.view(1, -1, 1, 1)
    y = y.permute(0, 2, 3, 1)
    return torch.relu(y) if relu else y


def _case(B, H, C, N, seed=0):
    from mlmicroservicetemplate_amd import ops

    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, H, H, C, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    return x, w, ops.pack_conv_weight(w), b


def _check(y, ref):
    err = (y.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
    assert err < 1e-2, err


SHAPES = [(32, 56, 64, 64), (32, 28, 128, 128), (32, 14, 256, 256), (32, 7, 512, 512)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"b{s[0]}h{s[1]}c{s[2]}")
@pytest.mark.parametrize("variant", range(12))
def test_pipe_variants_resnet_shapes(shape, variant):
    from mlmicroservicetemplate_amd import ops

    B, H, C, N = shape
    x, w, wp, b = _case(B, H, C, N)
    ref = _ref(x, w, b)
    ws = torch.empty(4 * B * H * H * N, device=DEV, dtype=torch.float32)
    for splitk in (1, 2, 4):
        if (C // 32) % splitk:
            continue
        for ipb in (1, 3):
            for _ in range(2):  # the counters of a split launch must be back at zero
                y = ops.conv3x3_pipe(x, wp, b, act=ops.ACT_RELU, variant=variant, splitk=splitk, ipb=ipb, workspace=ws)
                torch.cuda.synchronize()
                _check(y, ref)


@pytest.mark.parametrize("variant", [0, 1, 4, 5, 6, 9, 10])
def test_pipe_small_and_odd_batches(variant):
    from mlmicroservicetemplate_amd import ops

    for B, H, C, N in [(1, 56, 64, 64), (3, 28, 128, 96), (2, 14, 64, 64), (5, 7, 96, 64), (1, 7, 512, 512)]:
        if N % (64 if variant in (0, 3, 4, 6, 7, 8, 11) else 32):
            continue
        x, w, wp, b = _case(B, H, C, N, seed=B)
        y = ops.conv3x3_pipe(x, wp, b, act=ops.ACT_NONE, variant=variant)
        _check(y, _ref(x, w, b, relu=False))


def test_pipe_through_conv2d_cfg_and_graph():
    """The tuning-table route (cfg = CFG_PIPE + variant, splitk = ks + 16 * (ipb - 1)) inside a
    captured hipGraph, replayed."""
    from mlmicroservicetemplate_amd import ops

    x, w, wp, b = _case(32, 14, 256, 256)
    ref = _ref(x, w, b)
    ws = torch.empty(2 * 32 * 14 * 14 * 256, device=DEV, dtype=torch.float32)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())  # the inputs were made on the default stream
    with torch.cuda.stream(s):
        y = ops.conv2d_nhwc(x, wp, b, kernel=3, stride=1, pad=1, act=ops.ACT_RELU, workspace=ws,
                            cfg=ops.CFG_PIPE + 1, splitk=2 + 16)  # warm: counters allocated
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            y = ops.conv2d_nhwc(x, wp, b, kernel=3, stride=1, pad=1, act=ops.ACT_RELU, workspace=ws,
                                cfg=ops.CFG_PIPE + 1, splitk=2 + 16)
    for _ in range(3):
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        _check(y, ref)
