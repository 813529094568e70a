"""Batch split over concurrent HIP streams for the inference forwards (ViViT, TimeSformer, Swin3D).

Clips are independent and every kernel is batch-invariant, so the logits of a batch split into n parts
that run on n HIP streams (each part with its own workspace) are bit-identical to one stream; what the
split buys is overlap: one part's GEMM tail rounds and short launches run beside another part's
kernels (ViViT-B B = 8: 840 -> 916 clips/s with 2 streams, tools/exp_streams.py, round 3).
"""
from __future__ import annotations

import contextlib

import torch

# instrumentation switch (bench.py's per-kernel tables): every part of a split forward runs on the
# CALLER's stream, one after the other -- the headline's launches (same part sizes, kernels and
# workspaces) without the overlap, so HIP events around a launch time that launch alone
_SERIAL = [False]


@contextlib.contextmanager
def serial_parts(on: bool = True):
    prev = _SERIAL[0]
    _SERIAL[0] = bool(on)
    try:
        yield
    finally:
        _SERIAL[0] = prev


def serial() -> bool:
    return _SERIAL[0]


def split_bounds(B: int, ns: int, sizes=None) -> list:
    """Row bounds [0, b1, ..., B] of `ns` contiguous batch parts: `sizes` (clips per part, summing to B)
    or, when None, as even as possible (B * i // ns).  Raises ValueError on sizes that do not fit."""
    if sizes is None:
        return [B * i // ns for i in range(ns + 1)]
    sizes = [int(v) for v in sizes]
    if len(sizes) != ns or sum(sizes) != B or min(sizes) < 1:
        raise ValueError(f"split_sizes {sizes} must be {ns} positive part sizes summing to B={B}")
    return [sum(sizes[:i]) for i in range(ns + 1)]


def run_split(owner, x: torch.Tensor, ns: int, part_fn, num_labels: int, prepare=None) -> torch.Tensor:
    """part_fn(x_part, part_index, out=logits_rows) for each of `ns` contiguous batch parts, part i on
    owner._streams[i]; returns the [B, num_labels] logits (a buffer of `owner`, reused per call).

    `prepare()` builds the state every part reads (packed weights, bias caches) on the CALLER's
    stream before the fork: built inside part 0 on stream 0, it would be read by parts 1..n-1 on
    streams that wait only on the caller's stream (a cross-stream read-before-write), and the
    allocator would record those tensors on stream 0 alone."""
    dev = x.device
    if prepare is not None:
        prepare()
    B = x.shape[0]
    ns = max(1, min(int(ns), B))
    if owner._streams is None or len(owner._streams) < ns or owner._streams[0].device != dev:
        owner._streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
    key = (B, str(dev), "split_logits")
    if key not in owner._split_out:
        owner._split_out[key] = torch.zeros(B, num_labels, dtype=torch.float32, device=dev)
    logits = owner._split_out[key]
    cur = torch.cuda.current_stream(dev)
    bounds = split_bounds(B, ns, getattr(owner, "split_sizes", None))  # clips per part; None = as even as possible
    if _SERIAL[0]:
        for i in range(ns):
            part_fn(x[bounds[i]:bounds[i + 1]], i, out=logits[bounds[i]:bounds[i + 1]])
        return logits
    for i in range(ns):
        st = owner._streams[i]
        st.wait_stream(cur)
        x.record_stream(st)  # x may be freed by the caller while the side streams still read it
        with torch.cuda.stream(st):
            part_fn(x[bounds[i]:bounds[i + 1]], i, out=logits[bounds[i]:bounds[i + 1]])
    for i in range(ns):
        cur.wait_stream(owner._streams[i])
    return logits


class GraphReplay:
    """An inference forward captured once into a hipGraph (torch.cuda.CUDAGraph) and replayed.

    Static-input contract.  `key` = (the caller's input address, shape, strides, dtype, whatever
    selects the kernels: stream count, operand type, weights version); the first key's capture runs on
    the caller's own tensor, and a replay re-runs every kernel of the forward on the CURRENT contents
    of that tensor, so in-place updates of it are seen.  A caller that passes a NEW tensor of an
    already-captured shape (a DataLoader loop: one tensor per batch) does not recapture per batch:
    its input is copied into one internal static buffer per shape, captured once, and replayed.

    Each entry holds references to its input, the packed weights and the workspaces its kernels
    address (`keep()`, read after the capture: pass only this batch size's workspaces), so none of
    them is freed under it: torch.cuda.graph empties the allocator's cache when a capture starts, which
    unmaps freed blocks, so a graph whose buffers were merely dropped from a model cache would fault
    on replay after the next capture.  `run` returns the owner's logits buffer (overwritten by the
    next call), as the eager forward does."""

    def __init__(self, max_entries: int = 4):
        self.max_entries = max_entries
        self._entries = {}
        self.captures = 0

    def clear(self):
        self._entries = {}

    def _capture(self, key, x, forward, keep):
        if len(self._entries) >= self.max_entries:
            self._entries = {}
        dev = x.device
        cur = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            forward(x)  # first launches (kernel attributes), packing and workspaces outside the capture
        cur.wait_stream(side)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        # thread_local: HIP calls other threads make meanwhile (e.g. a process group's watchdog)
        # neither break this capture nor are broken by it.  A refused capture raises (measured:
        # after one, the next launch on the device fails too, so there is no eager fallback)
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            out = forward(x)
        self.captures += 1
        e = self._entries[key] = (g, out, x, (x,) + tuple(keep()))
        return e

    def run(self, key, x: torch.Tensor, forward, keep=lambda: ()):
        e = self._entries.get(key)
        if e is None:
            # key[1:] = everything but the input address: a new tensor of a captured configuration
            skey = ("static",) + tuple(key[1:])
            if skey in self._entries or any(k[0] != "static" and tuple(k[1:]) == tuple(key[1:]) for k in self._entries):
                e = self._entries.get(skey)
                if e is None:
                    e = self._capture(skey, torch.empty_like(x).copy_(x), forward, keep)
                else:
                    e[2].copy_(x)
                g, out, _, _ = e
                g.replay()
                return out
            e = self._capture(key, x, forward, keep)
        g, out, _, _ = e
        g.replay()
        return out
