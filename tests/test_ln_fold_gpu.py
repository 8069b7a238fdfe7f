"""LayerNorm folding in the tile GEMM (csrc/gemm_tile.hip "LayerNorm folding") vs fp32 PyTorch: the
folded projection, the residual / LN-residual epilogues with the output rows' statistics produced in
the launch, and BERT with / without the folding."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _rows(M, K, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    # non-zero per-row means and spreads, like a post-residual BERT stream
    h = torch.randn(M, K, device=DEV, generator=g) * (0.5 + torch.rand(M, 1, device=DEV, generator=g))
    h = h + 0.3 * torch.randn(M, 1, device=DEV, generator=g)
    return h.to(torch.bfloat16)


def _partials(t):
    """[M][W/128][2] per-128-column sums / sums of squares of the bf16 rows (what a PART epilogue writes)."""
    tf = t.float().view(t.shape[0], t.shape[1] // 128, 128)
    return torch.stack([tf.sum(2), (tf * tf).sum(2)], 2).reshape(-1).contiguous()


@pytest.mark.parametrize("M,N,K,cfg", [(4096, 2304, 768, 0), (1000, 3072, 768, 0), (4096, 768, 768, 16),
                                       (512, 768, 768, 5), (300, 512, 768, 4), (777, 2304, 768, 15)])
@pytest.mark.parametrize("act", ["none", "gelu"])
def test_folded_projection(M, N, K, cfg, act):
    """act(LN(h) @ W.T + b) from the raw rows h, the gamma-folded weight and h's row partials."""
    from mlmicroservicetemplate_amd import ops

    h = _rows(M, K, M + N)
    g = torch.Generator(device=DEV).manual_seed(3)
    w = (torch.randn(N, K, device=DEV, generator=g) / K**0.5).to(torch.bfloat16)
    b = 0.1 * torch.randn(N, device=DEV, generator=g)
    gam = (1 + 0.2 * torch.randn(K, device=DEV, generator=g)).to(torch.bfloat16).float()
    bet = (0.1 * torch.randn(K, device=DEV, generator=g)).to(torch.bfloat16).float()
    x = torch.nn.functional.layer_norm(h.float(), (K,), gam, bet, 1e-12)
    ref = x @ w.float().T + b
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    w2, c, b2 = ops.fold_layernorm(w, b, gam, bet)
    out = ops.gemm_tile_ln(h, w2, b2, act=act, fold_c=c, ln_part=_partials(h), cfg=cfg)
    assert rel(out, ref) < 2e-2, rel(out, ref)


@pytest.mark.parametrize("M,N,K,cfg", [(4096, 768, 3072, 0), (4096, 768, 768, 2), (333, 768, 3072, 15),
                                       (4096, 768, 3072, 10), (1000, 1024, 768, 4), (700, 768, 768, 5)])
@pytest.mark.parametrize("ln_res", [False, True])
def test_residual_epilogue_and_row_partials(M, N, K, cfg, ln_res):
    """a @ W.T + b + r with r = residual or LN(residual) (beta folded into the bias), and the output
    rows' partials written by the launch: they match the stored bf16 rows, and repeated launches are
    bit-identical."""
    from mlmicroservicetemplate_amd import ops

    g = torch.Generator(device=DEV).manual_seed(M + K)
    a = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) / K**0.5).to(torch.bfloat16)
    b = 0.1 * torch.randn(N, device=DEV, generator=g)
    r = _rows(M, N, 5)
    gam = 1 + 0.2 * torch.randn(N, device=DEV, generator=g)
    bet = 0.1 * torch.randn(N, device=DEV, generator=g)
    rf = r.float()
    if ln_res:
        kw, bias = dict(ln_part=_partials(r), ln_g=gam), b + bet
        resid = torch.nn.functional.layer_norm(rf, (N,), gam, bet, 1e-12)
    else:
        kw, bias, resid = {}, b, rf
    ref = a.float() @ w.float().T + b + resid
    part = ops.ln_partials(M, N, DEV)
    outs = []
    for _ in range(3):
        part.fill_(float("nan"))
        out = ops.gemm_tile_ln(a, w, bias, residual=r, stats_part=part, cfg=cfg, **kw)
        torch.cuda.synchronize()
        outs.append((out.clone(), part.clone()))
    assert rel(out, ref) < 2e-2, rel(out, ref)
    want = _partials(out)  # the statistics of the bf16 rows actually stored
    assert torch.allclose(part, want, rtol=1e-4, atol=1e-3)
    mu, rstd = ops.layernorm_from_partials(out, part)
    assert torch.allclose(mu, out.float().mean(1), atol=1e-4)
    for o, p_ in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(p_, outs[0][1])
    out2 = ops.gemm_tile_ln(a, w, bias, residual=r, cfg=cfg, **kw)  # no statistics requested
    assert torch.equal(out2, out)


def test_gemm_tile_ln_rejects_bad_args():
    from mlmicroservicetemplate_amd import ops

    a = torch.zeros(256, 768, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(768, 768, device=DEV, dtype=torch.bfloat16)
    c = torch.zeros(768, device=DEV)
    part = ops.ln_partials(256, 768, DEV)
    with pytest.raises(ValueError):
        ops.gemm_tile_ln(a, w, fold_c=c)  # folded form without the rows' statistics
    with pytest.raises(ValueError):
        ops.gemm_tile_ln(a, w, fold_c=c, ln_part=part, residual=a)
    with pytest.raises(ValueError):
        ops.gemm_tile_ln(a, w, residual=a, ln_part=part)  # no gamma
    with pytest.raises(ValueError):
        ops.gemm_tile_ln(a, w, residual=a, stats_part=part[:10])  # too small
    # an odd count of 128-column partials (width 640) cannot be read two per lane
    w640 = torch.zeros(640, 768, device=DEV, dtype=torch.bfloat16)
    r640 = torch.zeros(256, 640, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        ops.gemm_tile_ln(a, w640, residual=r640, ln_part=ops.ln_partials(256, 640, DEV), ln_g=torch.ones(640, device=DEV))
    a640 = torch.zeros(256, 640, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        ops.gemm_tile_ln(a640, torch.zeros(768, 640, device=DEV, dtype=torch.bfloat16), fold_c=c,
                         ln_part=ops.ln_partials(256, 640, DEV))


@pytest.mark.parametrize("B,S", [(8, 128), (32, 128)])
def test_bert_ln_fold_matches_unfolded_and_reference(B, S, monkeypatch):
    """The folded encoder (no LN kernel between the layers' GEMMs) against the unfolded one and fp32."""
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models import bert

    cfg = bert.BertConfig(num_labels=3)
    p = bert.init_bert(cfg, 0)
    torch.manual_seed(2)
    ids = torch.randint(1000, cfg.vocab, (B, S), device=DEV, dtype=torch.int32)
    tt = torch.zeros_like(ids)
    lens = torch.tensor(([128, 77, 10, 1] * (B // 4)), device=DEV, dtype=torch.int32)
    ref = bert.bert_reference({k: v.to(DEV) for k, v in p.items()}, ids, tt, lens, cfg)
    folded = bert.BertFused(p, DEV, cfg)
    assert folded.ln_fold
    monkeypatch.setenv("MLS_BERT_LN_FOLD", "0")
    plain = bert.BertFused(p, DEV, cfg)
    assert not plain.ln_fold
    calls = []
    real_ln = ops.layernorm
    monkeypatch.setattr(ops, "layernorm", lambda *a, **k: calls.append(a[0].shape[0]) or real_ln(*a, **k))
    out_f = folded(ids, tt, lens)[:, :3].float()
    # only the last layer's LayerNorms run as kernels, on the B [CLS] rows
    assert calls and all(n == B for n in calls), calls
    calls.clear()
    out_p = plain(ids, tt, lens)[:, :3].float()
    assert len(calls) == 2 * cfg.layers
    assert rel(out_f, ref) < 3e-2, rel(out_f, ref)
    assert rel(out_f, out_p) < 3e-2, rel(out_f, out_p)
