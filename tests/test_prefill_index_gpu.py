"""ops.prefill_slots / ops.last_rows (csrc/norm_ops.hip) -- the native replacements of the Llama
prefill's torch index arithmetic -- against the torch expressions they replace."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _ref_slots(pos, lens, B, S, slot_ids=None, table=None, page_rows=0, max_seq=0):
    b = torch.arange(B, device=pos.device, dtype=torch.int64).repeat_interleave(S)
    pl = pos.long()
    slot = slot_ids.long()[b] if slot_ids is not None else b
    valid = pl < lens.long()[b]
    if table is not None:
        p0 = torch.where(valid, pl, torch.zeros_like(pl))
        row = table.long()[slot, p0 // page_rows] * page_rows + p0 % page_rows
    else:
        row = slot * max_seq + pl
    return torch.where(valid, row, torch.full_like(pl, -1)).to(torch.int32)


@pytest.mark.parametrize("paged", [False, True])
@pytest.mark.parametrize("with_slots", [False, True])
def test_prefill_slots_matches_torch(paged, with_slots):
    from mlmicroservicetemplate_amd import ops

    g = torch.Generator().manual_seed(3)
    B, S, max_seq, page_rows, nslots = 5, 37, 256, 16, 12
    lens = torch.randint(1, S + 1, (B,), generator=g, dtype=torch.int32)
    start = torch.randint(0, 100, (B, 1), generator=g, dtype=torch.int32)
    pos = (start + torch.arange(S, dtype=torch.int32)).reshape(-1)
    lens = lens + start.reshape(-1)  # valid: pos < lens (a prompt continued at `start`)
    slot_ids = torch.randperm(nslots, generator=g)[:B].to(torch.int32) if with_slots else None
    table = torch.randperm(nslots * (max_seq // page_rows), generator=g).to(torch.int32).reshape(nslots, -1) if paged else None
    args = [t.to(DEV) if t is not None else None for t in (pos, lens, slot_ids, table)]
    got = ops.prefill_slots(args[0], args[1], B, S, args[2], table=args[3], page_rows=page_rows if paged else 0,
                            max_seq=0 if paged else max_seq)
    want = _ref_slots(*args[:2], B, S, args[2], args[3], page_rows, max_seq)
    torch.testing.assert_close(got, want, rtol=0, atol=0)
    assert (got == -1).any() and (got >= 0).any()


def test_last_rows_matches_index_select():
    from mlmicroservicetemplate_amd import ops

    B, S, D = 6, 19, 264
    x = torch.randn(B * S, D, device=DEV).to(torch.bfloat16)
    x2 = torch.randn(B * S, D, device=DEV).to(torch.bfloat16)
    lens = torch.tensor([1, 19, 7, 12, 3, 19], dtype=torch.int32, device=DEV)
    last = torch.arange(B, device=DEV) * S + lens.long() - 1
    assert torch.equal(ops.last_rows(x, lens, B, S), x.index_select(0, last))
    a, b = ops.last_rows(x, lens, B, S, x2)
    assert torch.equal(a, x.index_select(0, last)) and torch.equal(b, x2.index_select(0, last))
