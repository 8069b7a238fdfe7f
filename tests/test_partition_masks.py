"""CU-mask words of the engine's spatial partitions (ops.intra_partition_words, pure host code; the
device census that verifies them is tests/test_engine_gpu.py::test_cu_partition_masks_select_disjoint_halves)."""
import pytest

from mlmicroservicetemplate_amd.ops import intra_partition_words


def _bits(words):
    return {32 * i + j for i, w in enumerate(words) for j in range(32) if (w >> j) & 1}


@pytest.mark.parametrize("mode", ["intra", "intra_contig"])
@pytest.mark.parametrize("parts", [1, 2, 4, 8])
def test_partitions_are_disjoint_cover_and_keep_every_xcc(parts, mode):
    masks = intra_partition_words(parts, 256, mode)
    assert len(masks) == parts
    seen = set()
    for w in masks:
        bits = _bits(w)
        assert len(bits) == 256 // parts
        assert not (bits & seen)
        seen |= bits
        # bit b drives XCC b % 8: an XCC with no bit would run on ALL its CUs -> every XCC keeps a share
        per_xcc = [sum(1 for b in bits if b % 8 == x) for x in range(8)]
        assert per_xcc == [32 // parts] * 8
    assert seen == set(range(256))


def test_contiguous_halves_split_each_xcc_low_high():
    lo, hi = intra_partition_words(2, 256, "intra_contig")
    assert all(b // 8 < 16 for b in _bits(lo)) and all(b // 8 >= 16 for b in _bits(hi))
    ev, od = intra_partition_words(2, 256, "intra")
    assert all((b // 8) % 2 == 0 for b in _bits(ev)) and all((b // 8) % 2 == 1 for b in _bits(od))


def test_rejects_uneven_split():
    with pytest.raises(ValueError):
        intra_partition_words(3, 256)
