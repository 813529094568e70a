"""Batch split over concurrent HIP streams for the inference forwards (ViViT, TimeSformer, Swin3D).

Clips are independent and every kernel is batch-invariant, so the logits of a batch split into n parts
that run on n HIP streams (each part with its own workspace) are bit-identical to one stream; what the
split buys is overlap: one part's GEMM tail rounds and short launches run beside another part's
kernels (ViViT-B B = 8: 840 -> 916 clips/s with 2 streams, tools/exp_streams.py, round 3).
"""
from __future__ import annotations

import torch


def run_split(owner, x: torch.Tensor, ns: int, part_fn, num_labels: int) -> torch.Tensor:
    """part_fn(x_part, part_index, out=logits_rows) for each of `ns` contiguous batch parts, part i on
    owner._streams[i]; returns the [B, num_labels] logits (a buffer of `owner`, reused per call)."""
    dev = x.device
    B = x.shape[0]
    ns = max(1, min(int(ns), B))
    if owner._streams is None or len(owner._streams) < ns or owner._streams[0].device != dev:
        owner._streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
    key = (B, str(dev), "split_logits")
    if key not in owner._split_out:
        owner._split_out[key] = torch.zeros(B, num_labels, dtype=torch.float32, device=dev)
    logits = owner._split_out[key]
    cur = torch.cuda.current_stream(dev)
    bounds = [B * i // ns for i in range(ns + 1)]
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

    One entry per key (the caller's input address / shape / strides / dtype plus whatever selects
    the kernels: stream count, operand type, weights version).  A replay re-runs every kernel of
    the forward on the CURRENT contents of the input it was captured on, so in-place updates of
    that tensor are seen; the entry holds references to the input, the packed weights and the
    workspaces the graph's kernels address (`keep()`, read after the capture), so none of them is
    freed under it: torch.cuda.graph empties the allocator's cache when a capture starts, which
    unmaps freed blocks, so a graph whose buffers were merely dropped from a model cache would
    fault on replay after the next capture.  `run` returns the owner's logits buffer (overwritten by
    the next call), as the eager forward does."""

    def __init__(self, max_entries: int = 4):
        self.max_entries = max_entries
        self._entries = {}

    def clear(self):
        self._entries = {}

    def run(self, key, x: torch.Tensor, forward, keep=lambda: ()):
        e = self._entries.get(key)
        if e is None:
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
            e = self._entries[key] = (g, out, (x,) + tuple(keep()))
        g, out, _ = e
        g.replay()
        return out
