"""Host logic of the batch split over HIP streams (vclip_amd.streams.split_bounds, vivit.SPLIT_DEFAULT):
no GPU needed."""
import pytest

from vclip_amd import streams
from vclip_amd.vivit import SPLIT_DEFAULT


@pytest.mark.parametrize("B,ns,want", [(8, 2, [0, 4, 8]), (5, 2, [0, 2, 5]), (4, 4, [0, 1, 2, 3, 4]),
                                       (16, 3, [0, 5, 10, 16]), (1, 1, [0, 1])])
def test_even_split(B, ns, want):
    assert streams.split_bounds(B, ns) == want


@pytest.mark.parametrize("B,ns,sizes,want", [(8, 2, (5, 3), [0, 5, 8]), (8, 3, [1, 6, 1], [0, 1, 7, 8]),
                                             (3, 2, [2, 1], [0, 2, 3])])
def test_explicit_split(B, ns, sizes, want):
    assert streams.split_bounds(B, ns, sizes) == want


@pytest.mark.parametrize("B,ns,sizes", [(8, 2, [4, 3]), (8, 2, [8, 0]), (8, 3, [4, 4]), (8, 2, [9, -1])])
def test_bad_split_raises(B, ns, sizes):
    with pytest.raises(ValueError):
        streams.split_bounds(B, ns, sizes)


def test_vivit_default_split_covers_its_batch():
    """Every measured default (vivit.SPLIT_DEFAULT) is a valid split of its own batch, larger part first."""
    for (B, ns), sizes in SPLIT_DEFAULT.items():
        b = streams.split_bounds(B, ns, sizes)
        assert b[0] == 0 and b[-1] == B
        assert list(sizes) == sorted(sizes, reverse=True)
    assert SPLIT_DEFAULT[(8, 2)] == (5, 3)
