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


def test_pick_streams_rejects_priorities_of_the_wrong_length():
    """streams.pick_streams checks its priorities before touching a device."""
    with pytest.raises(ValueError):
        streams.pick_streams("cuda:0", 2, priorities=(0, 0, 0))
    assert streams.default_priorities(3) == (0, 0, 0)


def test_graph_replay_defaults():
    """Part graphs (streams.fork_parts) and the timed stream sets are the default; a fresh GraphReplay has
    no tuning record until it captures a split forward."""
    assert streams.PART_GRAPHS[0] is True
    assert streams.TUNE_CANDIDATES[0] >= 2
    assert streams.GraphReplay().tune_log is None


def test_fork_parts_runs_every_part_in_order_outside_a_capture():
    """Outside a capture fork_parts runs each part under its stream context, and the caller's stream waits
    for every part.  CPU stand-in streams record the calls."""
    calls = []

    class FakeStream:
        def __init__(self, name):
            self.name = name

        def wait_stream(self, other):
            calls.append(("wait", self.name, other.name))

    import contextlib
    orig = streams.torch.cuda.stream
    streams.torch.cuda.stream = lambda st: contextlib.nullcontext()
    try:
        a, b, cur = FakeStream("a"), FakeStream("b"), FakeStream("cur")
        streams.fork_parts([a, b], cur, [lambda: calls.append(("run", 0)), lambda: calls.append(("run", 1))])
    finally:
        streams.torch.cuda.stream = orig
    assert calls == [("wait", "a", "cur"), ("run", 0), ("wait", "b", "cur"), ("run", 1),
                     ("wait", "cur", "a"), ("wait", "cur", "b")]
