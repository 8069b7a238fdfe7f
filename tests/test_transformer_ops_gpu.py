"""Transformer kernels (K4 LN, K5 RMSNorm, K8 attention, K9 RoPE, K10 embeddings, K13 KV append)
vs the fp32 PyTorch oracles in ops.reference."""
import pytest
import torch

from mlmicroservicetemplate_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.fixture(scope="module")
def ops():
    from mlmicroservicetemplate_amd import ops as o

    o.lib()
    return o


@pytest.mark.parametrize("D", [64, 768, 1000, 2056, 4096, 8192])
@pytest.mark.parametrize("rms", [False, True])
def test_layernorm(ops, D, rms):
    torch.manual_seed(0)
    x = torch.randn(37, D, device=DEV).to(torch.bfloat16)
    r = torch.randn(37, D, device=DEV).to(torch.bfloat16)
    g = (torch.rand(D, device=DEV) + 0.5).to(torch.bfloat16)
    b = torch.randn(D, device=DEV).to(torch.bfloat16)
    res_out = torch.empty_like(x)
    y = ops.layernorm(x, g, None if rms else b, residual=r, residual_out=res_out, rms=rms, eps=1e-5)
    ref, hs = R.layernorm(x, g, None if rms else b, residual=r, eps=1e-5, rms=rms)
    assert rel(y, ref) < 2e-2
    assert rel(res_out, hs) < 1e-2
    y2 = ops.layernorm(x, g, None if rms else b, rms=rms)
    assert rel(y2, R.layernorm(x, g, None if rms else b, rms=rms)[0]) < 2e-2


def test_embed_ln_and_vocab_parallel(ops):
    torch.manual_seed(1)
    V, P, D, B, S = 1000, 128, 768, 3, 50
    word = torch.randn(V, D, device=DEV).to(torch.bfloat16)
    pos = torch.randn(P, D, device=DEV).to(torch.bfloat16)
    typ = torch.randn(2, D, device=DEV).to(torch.bfloat16)
    g = torch.ones(D, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros(D, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, V, (B * S,), device=DEV, dtype=torch.int32)
    tt = torch.randint(0, 2, (B * S,), device=DEV, dtype=torch.int32)
    y = ops.embed_layernorm(ids, tt, word, pos, typ, g, b, S, eps=1e-12)
    e = word[ids.long()].float() + pos[torch.arange(B * S, device=DEV) % S].float() + typ[tt.long()].float()
    ref = torch.nn.functional.layer_norm(e, (D,), eps=1e-12)
    assert rel(y, ref) < 2e-2
    # vocab shard [250, 500)
    out = ops.embedding(ids, word[250:500].contiguous(), lo=250, hi=500)
    inshard = ((ids >= 250) & (ids < 500)).unsqueeze(1)
    exp = torch.where(inshard, word[ids.long().clamp(0, V - 1)], torch.zeros_like(word[:1]))
    assert torch.equal(out, exp)


def test_rope_and_kv_append(ops):
    torch.manual_seed(2)
    T, Hq, Hkv, D = 45, 8, 2, 128
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    qkv0 = qkv.clone()
    pos = torch.randint(0, 1000, (T,), device=DEV, dtype=torch.int32)
    cos, sin = R.rope_tables(2048, D, 500000.0, DEV)
    ref_q = R.rope(qkv[:, : Hq * D].view(T, Hq, D), pos, cos, sin).reshape(T, -1)
    ref_k = R.rope(qkv[:, Hq * D: (Hq + Hkv) * D].view(T, Hkv, D), pos, cos, sin).reshape(T, -1)
    v_before = qkv[:, (Hq + Hkv) * D:].clone()
    ops.rope_(qkv, pos, cos, sin, Hq + Hkv, D)
    assert rel(qkv[:, : Hq * D], ref_q) < 1e-2
    assert rel(qkv[:, Hq * D: (Hq + Hkv) * D], ref_k) < 1e-2
    assert torch.equal(qkv[:, (Hq + Hkv) * D:], v_before)
    kc = torch.zeros(4 * 64, Hkv, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.randperm(4 * 64, device=DEV)[:T].to(torch.int32)
    ops.kv_append(qkv, Hq * D, (Hq + Hkv) * D, slots, kc, vc, Hkv, D)
    assert torch.equal(kc[slots.long()].reshape(T, -1), qkv[:, Hq * D: (Hq + Hkv) * D])
    assert torch.equal(vc[slots.long()].reshape(T, -1), qkv[:, (Hq + Hkv) * D:])
    # fused rope + append on a fresh copy matches the two-kernel path
    qkv2 = qkv0.clone()
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    ops.rope_kv_(qkv2, pos, cos, sin, Hq, Hkv, D, slots, kc2, vc2)
    assert torch.equal(qkv2, qkv) and torch.equal(kc2, kc) and torch.equal(vc2, vc)
    # slots derived in-kernel: 3 sequences x 15 positions into a [4][64] cache, padding skipped
    B, S, MS = 3, 15, 64
    pos3 = torch.arange(S, device=DEV, dtype=torch.int32).repeat(B)
    lens3 = torch.tensor([15, 7, 1], device=DEV, dtype=torch.int32)
    qkv3 = qkv0.clone()
    kc3, vc3 = torch.zeros_like(kc), torch.zeros_like(vc)
    ops.rope_kv_(qkv3, pos3, cos, sin, Hq, Hkv, D, None, kc3, vc3, lens=lens3, seq=S, max_seq=MS)
    kref = R.rope(qkv0[:, Hq * D: (Hq + Hkv) * D].view(T, Hkv, D), pos3, cos, sin).reshape(T, -1)
    for b in range(B):
        for p_ in range(S):
            row = kc3[b * MS + p_].reshape(-1)
            if p_ < int(lens3[b]):
                assert rel(row, kref[b * S + p_]) < 1e-2
                assert torch.equal(vc3[b * MS + p_].reshape(-1), qkv0[b * S + p_, (Hq + Hkv) * D:])
            else:
                assert not row.any()


@pytest.mark.parametrize("cfg", [
    # B, S, Hq, Hkv, D, causal, lens
    (3, 128, 12, 12, 64, False, [128, 77, 1]),
    (2, 77, 12, 12, 64, False, None),
    (4, 128, 12, 12, 64, False, [1, 64, 65, 127]),  # 8-wave BERT block: lens at the tile edges
    (2, 100, 4, 2, 64, True, None),                  # 8-wave block, causal + GQA
    (2, 200, 8, 2, 128, True, None),
    (1, 333, 4, 1, 128, True, None),
    (2, 64, 4, 1, 128, False, [64, 5]),
])
def test_flash_attention(ops, cfg):
    B, S, Hq, Hkv, D, causal, lens = cfg
    torch.manual_seed(3)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    kv_lens = torch.tensor(lens, device=DEV, dtype=torch.int32) if lens else None
    out = ops.flash_attention(qkv, B, S, Hq, Hkv, D, kv_lens=kv_lens, causal=causal)
    ref = R.attention(qkv, B, S, Hq, Hkv, D, kv_lens=kv_lens, causal=causal)
    assert rel(out, ref) < 2e-2


@pytest.mark.parametrize("q_rows", [1, 3, 16, 77, 128])  # 1-wave, 4-wave and 8-wave launches
def test_flash_attention_rows(ops, q_rows):
    """The first q_rows positions of each sequence (q from a strided [CLS]-style view, K/V from a
    fused [T, 2*Hkv*D] projection) vs the full reference attention's rows."""
    B, S, H, D = 4, 128, 12, 64
    torch.manual_seed(5)
    qkv = torch.randn(B * S, 3 * H * D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor([128, 90, 17, 1], device=DEV, dtype=torch.int32)
    ref = R.attention(qkv, B, S, H, H, D, kv_lens=lens).view(B, S, H * D)[:, :q_rows].reshape(B * q_rows, -1)
    rows = (torch.arange(B, device=DEV)[:, None] * S + torch.arange(q_rows, device=DEV)[None]).reshape(-1)
    wide = qkv[rows]  # [B*q_rows, 3HD]: q is its first H*D columns (row stride 3HD)
    kv = qkv[:, H * D:].contiguous()
    out = ops.flash_attention_rows(wide[:, : H * D], kv, B, S, q_rows, H, H, D, kv_lens=lens)
    assert out.shape == (B * q_rows, H * D)
    assert rel(out, ref) < 2e-2


@pytest.mark.parametrize("S,spike", [(256, 200), (128, 100)])  # 4-wave and 8-wave blocks
def test_flash_attention_spike_rescale(ops, S, spike):
    """Force the online-softmax rescale branch: one key row is a huge spike for every query,
    placed in a late tile so the running max jumps (guide §5.4 rule 26)."""
    B, H, D = 1, 2, 64
    torch.manual_seed(4)
    qkv = torch.randn(B * S, 3 * H * D, device=DEV)
    qkv[spike, H * D: 2 * H * D] = qkv[:, : H * D].mean(0) * 40  # key aligned with all queries
    qkv = qkv.to(torch.bfloat16)
    out = ops.flash_attention(qkv, B, S, H, H, D)
    ref = R.attention(qkv, B, S, H, H, D)
    assert rel(out, ref) < 2e-2


@pytest.mark.parametrize("Hq,Hkv,D", [(4, 1, 128), (32, 8, 128), (64, 8, 128), (8, 4, 128), (12, 12, 64)])
@pytest.mark.parametrize("chunk", [64, 128, 256])
@pytest.mark.parametrize("impl", ["valu", "mfma"])
def test_decode_attention(ops, Hq, Hkv, D, chunk, impl):
    if impl == "mfma" and D != 128:
        pytest.skip("matrix-core decode kernel: D = 128")
    torch.manual_seed(5)
    B, max_len = 4, 1024
    kc = torch.randn(B, max_len, Hkv, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, max_len, Hkv, D, device=DEV).to(torch.bfloat16)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    # one split (direct write), several splits (in-launch last-arriver merge), full cache
    lens = torch.tensor([1, 300, 1024, chunk], device=DEV, dtype=torch.int32)
    cnt = torch.zeros(B * Hkv, device=DEV, dtype=torch.int32)
    ref = R.decode_attention(q, kc, vc, lens, Hq, Hkv, D)
    for _ in range(3):  # the ticket counters must come back to zero between launches
        out = ops.decode_attention(q, kc, vc, lens, Hq, Hkv, D, chunk=chunk, counters=cnt, impl=impl)
        assert rel(out, ref) < 2e-2
    assert not cnt.any()


@pytest.mark.parametrize("impl,chunk", [("valu", 64), ("mfma", 256)])
def test_decode_attention_8k_context(ops, impl, chunk):
    """SURVEY K8's long end: one TP = 8 rank of Llama-3-8B (4 query heads, 1 KV head, D = 128)
    decoding against 8192-row caches (128 splits of 64 / 32 of 256)."""
    torch.manual_seed(6)
    B, max_len, Hq, Hkv, D = 2, 8192, 4, 1, 128
    kc = torch.randn(B, max_len, Hkv, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, max_len, Hkv, D, device=DEV).to(torch.bfloat16)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor([8192, 5001], device=DEV, dtype=torch.int32)
    cnt = torch.zeros(B * Hkv, device=DEV, dtype=torch.int32)
    ref = R.decode_attention(q, kc, vc, lens, Hq, Hkv, D)
    out = ops.decode_attention(q, kc, vc, lens, Hq, Hkv, D, chunk=chunk, counters=cnt, impl=impl)
    assert rel(out, ref) < 2e-2
    assert not cnt.any()


@pytest.mark.parametrize("cfg", [
    # B, S, Hq, Hkv, D, causal, lens, spike row
    (8, 512, 32, 8, 128, True, None, None),          # Llama-3-8B TP = 1 prefill shape
    (2, 200, 8, 2, 128, True, [200, 77], 150),       # partial last tile, padded sequence, late spike
    (3, 130, 4, 1, 128, False, [130, 64, 1], 100),   # bidirectional, lens at a tile edge / one key
    (1, 70, 4, 4, 128, True, None, 3),               # early spike, then tiles that must not rescale it away
    (32, 128, 12, 12, 64, False, None, None),        # BERT-base: one 8-wave block per (sequence, head)
    (4, 128, 12, 12, 64, False, [1, 64, 65, 127], 100),  # 8-wave block: lens at the tile edges
    (2, 100, 4, 2, 64, True, None, 50),              # 8-wave block, causal + GQA
])
def test_flash_attention_v2_matches_v1_and_fp32(ops, cfg):
    """The transposed-O prefill kernel (csrc/attention.hip flash_fwd2_kernel: lane-local rescale,
    per-lane row-sum partials, masks only on edge tiles, causal sub-tiles skipped; D = 128 4-wave
    and BERT's D = 64 8-wave blocks) vs the v1 kernel and the fp32 reference."""
    B, S, Hq, Hkv, D, causal, lens, spike = cfg
    torch.manual_seed(8)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV)
    if spike is not None:  # one key aligned with every query: the running max jumps at that tile
        qkv[spike, Hq * D: (Hq + Hkv) * D] = qkv[:, :D].mean(0).repeat(Hkv) * 40
    qkv = qkv.to(torch.bfloat16)
    kv_lens = torch.tensor(lens, device=DEV, dtype=torch.int32) if lens else None
    lib = ops.lib()
    old = lib.mls_flash_set_version(1)
    try:
        v1 = ops.flash_attention(qkv, B, S, Hq, Hkv, D, kv_lens=kv_lens, causal=causal)
        lib.mls_flash_set_version(2)
        v2 = ops.flash_attention(qkv, B, S, Hq, Hkv, D, kv_lens=kv_lens, causal=causal)
        torch.cuda.synchronize()
    finally:
        lib.mls_flash_set_version(old)
    ref = R.attention(qkv, B, S, Hq, Hkv, D, kv_lens=kv_lens, causal=causal)
    assert torch.isfinite(v2.float()).all()
    assert rel(v2, ref) < 2e-2
    assert rel(v2, v1) < 2e-2


def test_flash_attention_8k_causal(ops):
    """Causal prefill of an 8192-token prompt with the TP = 8 rank's head split."""
    torch.manual_seed(7)
    B, S, Hq, Hkv, D = 1, 8192, 4, 1, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    out = ops.flash_attention(qkv, B, S, Hq, Hkv, D, causal=True)
    ref = R.attention(qkv, B, S, Hq, Hkv, D, causal=True)
    assert rel(out, ref) < 2e-2


@pytest.mark.parametrize("Hq,Hkv", [(4, 1), (32, 8), (64, 8)])
@pytest.mark.parametrize("impl,chunk", [("valu", 64), ("mfma", 64), ("mfma", 128), ("mfma", 256)])
def test_decode_attention_rope_append(ops, Hq, Hkv, impl, chunk):
    """Rope mode == rope_kv_ (RoPE + append) followed by plain decode attention."""
    torch.manual_seed(6)
    B, max_len, D = 4, 512, 128
    kc = torch.randn(B, max_len, Hkv, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, max_len, Hkv, D, device=DEV).to(torch.bfloat16)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor([1, 77, 512, 129], device=DEV, dtype=torch.int32)
    pos = lens - 1
    cos, sin = R.rope_tables(max_len, D, 500000.0, DEV)
    kc2, vc2, qkv2 = kc.clone(), vc.clone(), qkv.clone()
    ops.rope_kv_(qkv2, pos, cos, sin, Hq, Hkv, D, None, kc2, vc2, lens=lens, seq=1, max_seq=max_len)
    ref = R.decode_attention(qkv2, kc2, vc2, lens, Hq, Hkv, D)
    out = ops.decode_attention(qkv, kc, vc, lens, Hq, Hkv, D, positions=pos, cos=cos, sin=sin, chunk=chunk, impl=impl)
    assert rel(out, ref) < 1e-2
    for b in range(B):
        p_ = int(pos[b])
        assert torch.equal(kc[b, p_], kc2[b, p_]) and torch.equal(vc[b, p_], vc2[b, p_])
