"""Fused ResNet-50 head (csrc/head.hip + the pooled epilogue of csrc/conv_gemm.hip) vs plain
PyTorch fp32 of the same bf16 operands: the average pool accumulated by the last conv, the
one-launch FC + softmax + top-k, the per-row error flags, the self-zeroing pool buffer, and the
whole model with the fused head against the unfused one."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("B", [1, 5, 32, 33])
def test_fc_head_matches_fp32(B):
    from mlmicroservicetemplate_amd import ops

    g = torch.Generator(device="cpu").manual_seed(B)
    pooled = (torch.rand(B, 2048, generator=g) * 2).to(DEV)
    w = (torch.randn(1000, 2048, generator=g) * 0.03).to(torch.bfloat16).to(DEV)
    b = (torch.randn(1000, generator=g) * 0.1).to(DEV)
    ref = pooled.to(torch.bfloat16).float() @ w.float().t() + b
    p0 = pooled.clone()
    vals, idx, logits = ops.fc_head(pooled, w, b, 5)
    torch.cuda.synchronize()
    assert (logits - ref).abs().max().item() < 2e-3 * ref.abs().max().item()
    assert pooled.abs().max().item() == 0.0  # zeroed for the next forward
    pr = torch.softmax(ref, -1)
    rv, ri = pr.topk(5, -1)
    top2 = ref.topk(2, -1).values
    sure = (top2[:, 0] - top2[:, 1]) > 1e-2
    assert torch.equal(idx[:, 0][sure].long(), ri[:, 0][sure])
    assert (vals - rv).abs().max().item() < 2e-3
    # the logits-only call (k = 0) on the same inputs
    pooled.copy_(p0)
    _, _, lg = ops.fc_head(pooled, w, b, 0)
    assert torch.equal(lg, logits)


@pytest.mark.parametrize("N,k", [(1000, 1), (1000, 5), (1000, 16), (1000, 17), (1000, 40), (10, 5), (300, 16)])
def test_fc_head_topk_against_torch(N, k):
    """The finisher's top-k (k <= 16: wave-local top-k + one-wave merge; larger k: block rounds)
    against torch.topk of the softmax of the logits the same launch returned."""
    from mlmicroservicetemplate_amd import ops

    B = 8
    g = torch.Generator(device="cpu").manual_seed(N + k)
    pooled = (torch.rand(B, 2048, generator=g) * 2).to(DEV)
    w = (torch.randn(N, 2048, generator=g) * 0.03).to(torch.bfloat16).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    vals, idx, logits = ops.fc_head(pooled, w, b, k)
    torch.cuda.synchronize()
    rv, ri = torch.softmax(logits.float(), -1).topk(k, -1)
    assert torch.allclose(vals.float(), rv, rtol=1e-4, atol=1e-7)
    distinct = torch.ones_like(rv, dtype=torch.bool)
    distinct[:, 1:] &= rv[:, 1:] != rv[:, :-1]
    distinct[:, :-1] &= rv[:, :-1] != rv[:, 1:]
    assert torch.equal(idx.long()[distinct], ri[distinct])
    assert (idx >= 0).all() and (idx < N).all()


def test_fc_head_error_rows_and_repeat():
    from mlmicroservicetemplate_amd import ops

    B = 32
    w = (torch.randn(1000, 2048, device=DEV) * 0.03).to(torch.bfloat16)
    b = torch.zeros(1000, device=DEV)
    err = torch.zeros(B, dtype=torch.int32, device=DEV)
    err[3] = 1
    err[31] = 1
    for it in range(3):  # the arrival counters reset themselves
        pooled = torch.rand(B, 2048, device=DEV)
        ref = (pooled.to(torch.bfloat16).float() @ w.float().t()).argmax(-1)
        vals, idx, _ = ops.fc_head(pooled, w, b, 5, err=err)
        torch.cuda.synchronize()
        assert idx[3].tolist() == [-1] * 5 and idx[31].tolist() == [-1] * 5
        assert torch.isnan(vals[3]).all() and torch.isnan(vals[31]).all()
        ok = torch.ones(B, dtype=torch.bool, device=DEV)
        ok[3] = ok[31] = False
        assert (idx[ok, 0].long() == ref[ok]).float().mean().item() > 0.9
        assert torch.isfinite(vals[ok]).all()


def test_fc_head_graph_survives_larger_eager_call_on_its_stream():
    """A graph captured with a small head (engine A) keeps working after a larger head runs eagerly
    on the SAME stream (engine B warming up on a pooled masked stream): the partial slabs come
    from each call's own workspace tensor (the graph's from its pool), so nothing the graph
    captured is freed or re-sized under it (round-5 advisor finding on head_slabs)."""
    from mlmicroservicetemplate_amd import ops

    g = torch.Generator(device="cpu").manual_seed(7)
    w = (torch.randn(1000, 2048, generator=g) * 0.03).to(torch.bfloat16).to(DEV)
    b = (torch.randn(1000, generator=g) * 0.1).to(DEV)
    small = (torch.rand(8, 2048, generator=g) * 2).to(DEV)
    src = small.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        vals0, idx0, lg0 = ops.fc_head(small, w, b, 5)  # eager reference (zeroes `small`)
        small.copy_(src)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            gv, gi, glg = ops.fc_head(small, w, b, 5)
        small.copy_(src)
        big = (torch.rand(64, 2048, generator=g) * 2).to(DEV)
        ops.fc_head(big, w, b, 5)  # a larger eager call on the same stream
        junk = torch.full((64 * 8 * 1000,), 7.0, device=DEV)  # reuse pressure on freed memory
        for _ in range(2):
            small.copy_(src)
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(gi, idx0) and torch.equal(glg, lg0)
        del junk


def test_conv2d_pool_matches_fp32():
    from mlmicroservicetemplate_amd import ops

    B, H, C, N = 32, 7, 512, 2048
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(B, H, H, C, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, C, 1, 1, generator=g) * (2 / C) ** 0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    res = torch.randn(B, H, H, N, generator=g).to(torch.bfloat16).to(DEV)
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w.float()) + bias.view(1, -1, 1, 1) + res.permute(0, 3, 1, 2).float()
    ref = torch.relu(y).mean(dim=(2, 3))
    wp = ops.pack_conv_weight(w)
    for cfg in (0, 9, 12, 4):
        pool = torch.zeros(B, N, device=DEV)
        out = ops.conv2d_pool(x, wp, bias, pool, kernel=1, residual=res, act=ops.ACT_RELU, cfg=cfg)
        torch.cuda.synchronize()
        assert out is None
        err = (pool - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-2, (cfg, err)
    # with the output written as well
    pool = torch.zeros(B, N, device=DEV)
    out = ops.conv2d_pool(x, wp, bias, pool, kernel=1, residual=res, act=ops.ACT_RELU, pool_only=False)
    torch.cuda.synchronize()
    assert (out.float() - torch.relu(y).permute(0, 2, 3, 1)).abs().max().item() < 0.05 * y.abs().max().item()


def test_resnet_fused_head_vs_unfused_and_graph():
    from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50, resnet50_reference
    from mlmicroservicetemplate_amd.ops import autotune

    params = init_resnet50(0)
    tuning = autotune.load_tuning("resnet50", 32)
    m = ResNet50Fused(params, DEV, max_batch=32, tuning=tuning)
    assert m.fuse_head
    imgs = torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8, device=DEV)
    ref = resnet50_reference({k: v.to(DEV) for k, v in params.items()}, imgs).float()
    s = torch.cuda.Stream()
    # the model's weight packing, the images and the reference ran on the default stream: order
    # the side stream after them (without this the first forward raced the packing kernels)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        lg = m(imgs).float()
        v1, i1 = m.classify(imgs, 5)
        v2, i2 = m.classify(imgs, 5)  # the pool buffer was re-zeroed: identical results
        torch.cuda.synchronize()
        assert torch.equal(i1, i2) and torch.equal(v1, v2)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            gv, gi = m.classify(imgs, 5)
        for _ in range(2):
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(gi, i1)
    rel = ((lg - ref).abs().max() / ref.abs().max()).item()
    assert rel < 3e-2, rel
    top2 = ref.topk(2, -1).values
    sure = (top2[:, 0] - top2[:, 1]) / ref.abs().max() > 1e-2
    assert torch.equal(i1[:, 0][sure].long(), ref.argmax(-1)[sure])
    os.environ["MLS_FUSED_HEAD"] = "0"
    try:
        mu = ResNet50Fused(params, DEV, max_batch=32, tuning=tuning)
    finally:
        del os.environ["MLS_FUSED_HEAD"]
    assert not mu.fuse_head
    vu, iu = mu.classify(imgs, 5)
    torch.cuda.synchronize()
    assert torch.equal(iu[:, 0][sure], i1[:, 0][sure])
    # probabilities against the fp32 reference at the returned classes: the fused head (fp32 pool
    # sums, one bf16 rounding) must be at least as close as the unfused one (bf16 pool output)
    pref = torch.softmax(ref, -1)
    ef = (v1 - pref.gather(1, i1.long())).abs().max().item()
    eu = (vu - pref.gather(1, iu.long())).abs().max().item()
    assert ef < 5e-2 and ef <= eu + 1e-2, (ef, eu)
