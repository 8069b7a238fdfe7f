"""Paged KV cache on the GPU: the decode-attention kernel through a page table equals the same
kernel on the contiguous cache (plain and RoPE + append mode), and the fused Llama generates the
same tokens with a paged pool as with per-slot caches (lockstep generate and continuous batching)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _paged_copy(cache, pages_per_seq, num_pages, perm_seed=0):
    """[B, L, Hkv, D] contiguous cache -> (pool [num_pages, 64, Hkv, D], table [B, pages_per_seq])
    with the sequence pages scattered over the pool in a random order (page 0 left as scratch)."""
    B, L, Hkv, D = cache.shape
    g = torch.Generator().manual_seed(perm_seed)
    order = (torch.randperm(num_pages - 1, generator=g) + 1)[: B * pages_per_seq]
    table = order.view(B, pages_per_seq).to(torch.int32)
    pool = torch.zeros(num_pages, 64, Hkv, D, device=cache.device, dtype=cache.dtype)
    for b in range(B):
        for p in range(pages_per_seq):
            pool[int(table[b, p])] = cache[b, p * 64:(p + 1) * 64]
    return pool, table.to(cache.device)


@pytest.mark.parametrize("Hq,Hkv", [(4, 1), (32, 8)])
@pytest.mark.parametrize("impl", ["valu", "mfma"])
def test_paged_decode_attention_equals_contiguous(Hq, Hkv, impl, monkeypatch):
    from mlmicroservicetemplate_amd import ops

    monkeypatch.setenv("MLS_DECODE_ATTN", impl)

    torch.manual_seed(9)
    B, L, D = 3, 512, 128
    kc = torch.randn(B, L, Hkv, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor([1, 200, 512], device=DEV, dtype=torch.int32)
    kp, table = _paged_copy(kc, L // 64, 40, 1)
    vp, _ = _paged_copy(vc, L // 64, 40, 1)
    want = ops.decode_attention(q, kc, vc, lens, Hq, Hkv, D, chunk=64)
    got = ops.decode_attention(q, kp, vp, lens, Hq, Hkv, D, chunk=64, page_table=table)
    assert torch.equal(got, want)


@pytest.mark.parametrize("impl", ["valu", "mfma"])
def test_paged_decode_attention_rope_append(impl, monkeypatch):
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops import reference as R

    monkeypatch.setenv("MLS_DECODE_ATTN", impl)

    torch.manual_seed(10)
    B, L, Hq, Hkv, D = 3, 256, 32, 8, 128
    kc = torch.randn(B, L, Hkv, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor([1, 130, 256], device=DEV, dtype=torch.int32)
    pos = lens - 1
    cos, sin = R.rope_tables(L, D, 500000.0, DEV)
    kp, table = _paged_copy(kc, L // 64, 20, 2)
    vp, _ = _paged_copy(vc, L // 64, 20, 2)
    want = ops.decode_attention(qkv, kc, vc, lens, Hq, Hkv, D, positions=pos, cos=cos, sin=sin)
    got = ops.decode_attention(qkv, kp, vp, lens, Hq, Hkv, D, positions=pos, cos=cos, sin=sin, page_table=table)
    assert torch.equal(got, want)
    for b in range(B):  # the appended row landed in the right page
        p_ = int(pos[b])
        page = int(table[b, p_ // 64])
        assert torch.equal(kp[page, p_ % 64], kc[b, p_]) and torch.equal(vp[page, p_ % 64], vc[b, p_])


def test_paged_decode_rejects_bad_geometry():
    from mlmicroservicetemplate_amd import ops

    kc = torch.zeros(4, 32, 1, 128, device=DEV, dtype=torch.bfloat16)  # 32-row pages != chunk 64
    q = torch.zeros(1, 6 * 128, device=DEV, dtype=torch.bfloat16)
    lens = torch.ones(1, device=DEV, dtype=torch.int32)
    with pytest.raises(ValueError):
        ops.decode_attention(q, kc, kc, lens, 4, 1, 128, chunk=64,
                             page_table=torch.zeros(1, 2, device=DEV, dtype=torch.int32))


def test_fused_llama_paged_matches_contiguous():
    from mlmicroservicetemplate_amd.models.llama import GenParams, LlamaTP, init_llama_shard, tiny_config
    from mlmicroservicetemplate_amd.models.llama_serving import ContinuousLlama

    cfg = tiny_config(layers=2, hidden=512, heads=8, kv_heads=2, head_dim=128, intermediate=1024)
    p = init_llama_shard(cfg, 1, 0, seed=5, device=DEV)
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(3, 2000, (3, 90), generator=g)
    lens = torch.tensor([90, 33, 4])
    gp = GenParams(max_new_tokens=10)
    want = LlamaTP(p, cfg, backend="fused", device=DEV, max_batch=4, max_seq=256).generate(ids, lens, gp)
    paged = LlamaTP(p, cfg, backend="fused", device=DEV, max_batch=4, max_seq=256, kv_pages=9)
    got = paged.generate(ids, lens, gp)
    assert torch.equal(got, want)
    # continuous batching over the paged pool: 8 data pages, requests of 2 pages each
    eng = ContinuousLlama(paged)
    futs = [eng.submit(ids[b, : int(lens[b])].tolist(), gp) for b in range(3)]
    eng.start()  # all three admitted by the first iteration: the same [3, 90] prefill as generate()
    outs = [f.result(timeout=120) for f in futs]
    eng.stop()
    eos = set(cfg.eos_ids)
    for b in range(3):
        w = want[b].tolist()
        cut = next((i + 1 for i, t in enumerate(w) if t in eos), len(w))
        assert outs[b] == w[:cut]
    assert paged.pages.free_pages == 8


def test_fused_llama_fp8_decode_close_to_bf16(monkeypatch):
    """MLS_DECODE_FP8=1: decode steps run the W8A8 kernel (counted) and their top logits stay within
    fp8 error of the bf16 model's."""
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.llama import LlamaTP, init_llama_shard, tiny_config

    cfg = tiny_config(layers=2, hidden=512, heads=8, kv_heads=2, head_dim=128, intermediate=1024)
    p = init_llama_shard(cfg, 1, 0, seed=6, device=DEV)
    ref = LlamaTP(p, cfg, backend="fused", device=DEV, max_batch=2, max_seq=128)
    monkeypatch.setenv("MLS_DECODE_FP8", "1")
    monkeypatch.setenv("MLS_DECODE_FP8_MIN", "0")  # the tiny model's matrices are all small
    q8 = LlamaTP(p, cfg, backend="fused", device=DEV, max_batch=2, max_seq=128)
    assert q8.fp8
    calls = {"n": 0}
    real = ops.skinny_fp8

    def counting(*a, **k):
        calls["n"] += 1
        return real(*a, **k)

    monkeypatch.setattr(ops, "skinny_fp8", counting)
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(3, 2000, (2, 20), generator=g).to(DEV).to(torch.int32)
    lens = torch.tensor([20, 11], device=DEV, dtype=torch.int32)
    pos = torch.arange(20, device=DEV, dtype=torch.int32).unsqueeze(0).expand(2, 20).contiguous()
    for m in (ref, q8):
        m.use_graphs = False  # eager decode so the counter sees the calls
        m.step(ids, pos, lens, decode=False, k=5)
    tok = torch.tensor([[7], [9]], device=DEV, dtype=torch.int32)
    cur = lens.view(2, 1).clone()
    v_ref, i_ref = ref.decode_step(tok, cur, 5, max_ctx=21)
    v_q8, i_q8 = q8.decode_step(tok, cur, 5, max_ctx=21)
    assert calls["n"] >= 2 * cfg.layers
    assert ((v_q8 - v_ref).abs().max() / v_ref.abs().max()).item() < 0.1


@pytest.mark.parametrize("paged", [False, True])
@pytest.mark.parametrize("impl", ["valu", "mfma"])
def test_head_major_decode_equals_row_major(paged, impl, monkeypatch):
    """Head-major caches ([B, Hkv, L, D] / paged [pages, Hkv, 64, D]) give the row-major result bit
    for bit, plain and in RoPE + append mode (the appended row lands in the head-major slot)."""
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops import reference as R

    monkeypatch.setenv("MLS_DECODE_ATTN", impl)
    torch.manual_seed(11)
    B, L, Hq, Hkv, D = 3, 256, 32, 8, 128
    kc = torch.randn(B, L, Hkv, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor([1, 130, 256], device=DEV, dtype=torch.int32)
    pos = lens - 1
    cos, sin = R.rope_tables(L, D, 500000.0, DEV)
    for rope in (False, True):
        kw = dict(positions=pos, cos=cos, sin=sin) if rope else {}
        k1, v1 = kc.clone(), vc.clone()
        if paged:
            kp, table = _paged_copy(k1, L // 64, 20, 3)
            vp, _ = _paged_copy(v1, L // 64, 20, 3)
            want = ops.decode_attention(qkv, kp, vp, lens, Hq, Hkv, D, page_table=table, **kw)
            kh, vh = kp.new_zeros(20, Hkv, 64, D), vp.new_zeros(20, Hkv, 64, D)
            kh.copy_(_paged_copy(kc, L // 64, 20, 3)[0].permute(0, 2, 1, 3))
            vh.copy_(_paged_copy(vc, L // 64, 20, 3)[0].permute(0, 2, 1, 3))
            got = ops.decode_attention(qkv, kh, vh, lens, Hq, Hkv, D, page_table=table, head_major=True, **kw)
            if rope:
                assert torch.equal(kh.permute(0, 2, 1, 3), kp) and torch.equal(vh.permute(0, 2, 1, 3), vp)
        else:
            want = ops.decode_attention(qkv, k1, v1, lens, Hq, Hkv, D, **kw)
            kh = kc.permute(0, 2, 1, 3).contiguous()
            vh = vc.permute(0, 2, 1, 3).contiguous()
            got = ops.decode_attention(qkv, kh, vh, lens, Hq, Hkv, D, head_major=True, **kw)
            if rope:
                assert torch.equal(kh.permute(0, 2, 1, 3), k1) and torch.equal(vh.permute(0, 2, 1, 3), v1)
        assert torch.equal(got, want)


def test_head_major_writers():
    """rope_kv_ / kv_append with hm_rows write the same rows as the row-major layout."""
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops import reference as R

    torch.manual_seed(12)
    T, Hq, Hkv, D, MS = 6, 8, 2, 128, 128
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    slots = torch.tensor([0, 5, 127, 128, 200, -1], device=DEV, dtype=torch.int32)
    pos = torch.tensor([0, 5, 127, 0, 72, 3], device=DEV, dtype=torch.int32)
    cos, sin = R.rope_tables(256, D, 500000.0, DEV)
    for R_ in (64, MS):
        kr = torch.zeros(2 * MS, Hkv, D, device=DEV, dtype=torch.bfloat16)
        vr = torch.zeros_like(kr)
        kh = torch.zeros(2 * MS // R_, Hkv, R_, D, device=DEV, dtype=torch.bfloat16)
        vh = torch.zeros_like(kh)
        ops.kv_append(qkv, Hq * D, (Hq + Hkv) * D, slots, kr, vr, Hkv, D)
        ops.kv_append(qkv, Hq * D, (Hq + Hkv) * D, slots, kh, vh, Hkv, D, hm_rows=R_)
        assert torch.equal(kh.permute(0, 2, 1, 3).reshape(-1, Hkv, D), kr)
        assert torch.equal(vh.permute(0, 2, 1, 3).reshape(-1, Hkv, D), vr)
        q1, q2 = qkv.clone(), qkv.clone()
        kr.zero_(), vr.zero_(), kh.zero_(), vh.zero_()
        ops.rope_kv_(q1, pos, cos, sin, Hq, Hkv, D, slots, kr, vr)
        ops.rope_kv_(q2, pos, cos, sin, Hq, Hkv, D, slots, kh, vh, hm_rows=R_)
        assert torch.equal(q1, q2)
        assert torch.equal(kh.permute(0, 2, 1, 3).reshape(-1, Hkv, D), kr)
