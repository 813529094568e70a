"""Batch split over concurrent HIP streams for the inference forwards (ViViT, TimeSformer, Swin3D).

Clips are independent and every kernel is batch-invariant, so the logits of a batch split into n parts
that run on n HIP streams (each part with its own workspace) are bit-identical to one stream; what the
split buys is overlap: one part's GEMM tail rounds and short launches run beside another part's
kernels (ViViT-B B = 8: 840 -> 916 clips/s with 2 streams, tools/exp_streams.py, round 3).
"""
from __future__ import annotations

import contextlib
import time

import torch

from . import ops

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


# Part streams (round 6).  Whether the parts of a split forward overlap depends on the streams they run on:
#  * streams on ONE hardware queue serialize.  HIP maps streams onto a few queues per process
#    (GPU_MAX_HW_QUEUES, 4 here) and which of torch's pool streams share one depends on how many streams
#    the process made before (tools/hwq_probe.py: of six consecutive pool streams, three pairs shared).
#    pick_streams measures (two probes, see there);
#  * beyond that, through state no probe here predicted: with every pair on different queues the ViViT-B
#    B = 8 5 + 3-clip forward ran 850-900 or 960-1000 clips/s from one stream set to the next, ResNet3D-50
#    990 or 1517, TimeSformer-B 1430 or 1829, each set stable over repeated replays in its process
#    (tools/exp_vivit_hwq.py, tools/ab_stream_modes.py; priorities did not decide it either, and a probe
#    of whether one queue's dispatch waits for the other's, tools/hwq_pipe_probe.py, did not predict it).
#    So GraphReplay times the captured part graphs, and part_streams the eager forward, on several picked
#    stream sets and keep the fastest.
# The picked set is cached per (device, priorities).
_PICKED = {}
PICK_STATUS = {}  # (device, priorities) -> True when every picked pair measured concurrent


def default_priorities(n: int) -> tuple:
    return (0,) * n


def _spin_time(sts, iters, device):
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for st in sts:
        with torch.cuda.stream(st):
            ops.spin(iters, device)
    torch.cuda.synchronize(device)
    return time.perf_counter() - t0


def _calibrate(device):
    """(iters, seconds) of a one-wave vc_spin of at least 0.5 ms on the current stream"""
    cur = [torch.cuda.current_stream(device)]
    iters = 16
    _spin_time(cur, iters, device)  # first launch: kernel load
    while iters < (1 << 16) and _spin_time(cur, iters, device) < 5e-4:
        iters *= 2
    return iters, min(_spin_time(cur, iters, device) for _ in range(3))


def _behind(a, b, device, blocks: int, iters: int = 24) -> float:
    """Completion time of a one-workgroup spin on stream b queued right after a `blocks`-workgroup spin
    (four rounds of the GPU's wave slots) on stream a, over a's: ~0.3 when b's workgroup is dispatched
    beside a's, ~0.96 when b waits for a's whole dispatch (best of two; tools/hwq_pipe_probe.py)."""
    best = 9.0
    for _ in range(2):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        with torch.cuda.stream(a):
            ops.spin(iters, device, blocks)
        with torch.cuda.stream(b):
            ops.spin(1, device, 1)
        b.synchronize()
        tb = time.perf_counter() - t0
        a.synchronize()
        best = min(best, tb / (time.perf_counter() - t0))
    return best


def pick_streams(device, n: int, priorities=None, candidates: int = 12, fresh: bool = False, against=()) -> list:
    """`n` streams of torch's pool, stream i at priority priorities[i] (default_priorities(n) when None),
    every pair among them and with each stream of `against` (e.g. the caller's stream, when it runs work
    beside them) measured to run side by side; cached unless `fresh` (a new set from the next pool
    streams, for GraphReplay._tune).  Falls back to unmeasured candidates (PICK_STATUS False) when no
    such set turns up, and to fresh pool streams while a graph capture is running (no synchronisation).

    Two probes: (1) a one-wave spin on each of two streams takes one spin's time when they sit on
    different hardware queues and two when they share one; (2) a one-workgroup spin queued behind a
    four-round spin on the other stream finishes after the first round (0.3 of it) unless the two
    queues are dispatched one kernel at a time (0.96).  The ViViT-B train step ran 183 clips/s with
    its weight-gradient stream in relation (2) to the main stream and 206 with the two side streams
    so, 219-222 in every trial with all pairs at 0.3 (tools/exp_train_streams.py, twelve trials)."""
    device = torch.device(device)
    prios = tuple(int(p) for p in (default_priorities(n) if priorities is None else priorities))
    if len(prios) != n:
        raise ValueError(f"pick_streams: {len(prios)} priorities for {n} streams")
    against = tuple(against)
    key = (device.index, prios) + ((tuple(s.cuda_stream for s in against),) if against else ())
    got = None if fresh else _PICKED.get(key)
    if got is not None:
        return got
    if n <= 1 and not against or torch.cuda.is_current_stream_capturing():
        return [torch.cuda.Stream(device=device, priority=p) for p in prios]
    cur = [torch.cuda.current_stream(device)]
    iters, one = _calibrate(device)
    blocks = 4 * 32 * torch.cuda.get_device_properties(device).multi_processor_count
    _behind(torch.cuda.Stream(device=device), cur[0], device, blocks)

    def fits(c, q):
        return (min(_spin_time([q, c], iters, device) for _ in range(2)) < 1.5 * one
                and _behind(q, c, device, blocks) < 0.6 and _behind(c, q, device, blocks) < 0.6)

    picked, ok = [], True
    for p in prios:
        cands = [torch.cuda.Stream(device=device, priority=p) for _ in range(candidates)]
        for c in cands:
            if all(fits(c, q) for q in list(against) + picked):
                picked.append(c)
                break
        else:
            picked.append(cands[0])
            ok = False
    if not fresh:  # PICK_STATUS / _PICKED describe the cached set only
        PICK_STATUS[key] = ok
        _PICKED[key] = picked
    return picked


# A/B switch: False captures a split forward as ONE graph holding every part's branch (rounds 2-5)
PART_GRAPHS = [True]
# stream sets GraphReplay._tune times the part graphs on (1: the capture's own, no tuning)
TUNE_CANDIDATES = [6]
# priority patterns of the fresh candidate sets, in rotation: (part index, part count) -> priority
TUNE_PRIORITIES = [lambda i, n: 0, lambda i, n: -1 if i == 0 else 0]

# set by GraphReplay while it captures a split forward: fork_parts then captures each part into a graph of
# its own (stream, graph) instead of running it
_PART_CAPTURE = [None]


def fork_parts(sts, cur, fns) -> None:
    """fns[i]() on stream sts[i] after everything queued on `cur`; `cur` then waits for every part.
    Under GraphReplay's capture each part becomes a graph of its own, replayed on its own stream: one
    graph holding both branches runs them on queues HIP picks at instantiation, which serialized the
    parts in about half the processes (tools/exp_vivit_hwq.py)."""
    cap = _PART_CAPTURE[0]
    for st, fn in zip(sts, fns):
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            if cap is None:
                fn()
            else:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st, capture_error_mode="thread_local"):
                    fn()
                cap.append((st, g))
    for st in sts:
        cur.wait_stream(st)


def _rank_sets(cands, run, device):
    """Time run(streams) on every candidate stream set: three warm-up runs of the first (the clock ramps up
    over the first launches of a fresh process), then two passes in opposite orders (a drifting clock
    favours no position) of one untimed and two timed runs per set.  Returns (index of the set with the
    lowest second-best of its four times, [that time per set])."""
    for _ in range(3):
        run(cands[0])
    ts = [[] for _ in cands]
    for rnd in range(2):
        for i in (range(len(cands)) if rnd == 0 else reversed(range(len(cands)))):
            run(cands[i])
            for _ in range(2):
                torch.cuda.synchronize(device)
                t0 = time.perf_counter()
                run(cands[i])
                torch.cuda.synchronize(device)
                ts[i].append(time.perf_counter() - t0)
    score = [sorted(t)[1] for t in ts]
    return min(range(len(cands)), key=lambda i: score[i]), score


def _candidate_sets(device, n, first):
    """`first` and TUNE_CANDIDATES - 1 fresh pick_streams sets, priority patterns TUNE_PRIORITIES in rotation"""
    pats = [tuple(p(i, n) for i in range(n)) for p in TUNE_PRIORITIES]
    return [list(first)] + [pick_streams(device, n, pats[t % len(pats)], fresh=True)
                            for t in range(TUNE_CANDIDATES[0] - 1)]


# eager split forwards tune their part streams on the first call per configuration (EAGER_TUNE); _NO_TUNE > 0
# while GraphReplay runs a forward for its own purposes (its warm-up and part-capture passes)
EAGER_TUNE = [True]
_NO_TUNE = [0]


def part_streams(owner, key, n: int, run, device, priorities=None) -> list:
    """The part streams of an eager split forward.  Explicit `priorities` (an A/B hook): pick_streams of
    those.  Otherwise, on the first call per `key`, the forward itself (`run(streams)` enqueues it on a
    stream set) is timed on the sets _candidate_sets gives and the fastest is kept for this owner and key
    (`owner.eager_tune_log`: (priorities, ms) per set); later calls reuse it.  Untuned (the cached
    pick_streams set) while instrumented (serial parts, an op recorder, kernel events), inside a capture,
    or under _NO_TUNE.  The eager ViViT-B B = 8 two-stream forward ran 850-885 clips/s instead of
    930-970 in about one process in five on the cached pick alone (tools/exp_vivit_hwq.py)."""
    if priorities is not None:
        return pick_streams(device, n, tuple(priorities)[:n])
    cache = owner.__dict__.setdefault("_eager_sets", {})
    got = cache.get(key)
    if got is not None:
        return got
    base = pick_streams(device, n)
    if (n <= 1 or not EAGER_TUNE[0] or _NO_TUNE[0] or _SERIAL[0] or ops._REC[0] is not None
            or getattr(owner, "kernel_events", None) is not None or torch.cuda.is_current_stream_capturing()):
        return base
    cands = _candidate_sets(device, n, base)
    k, score = _rank_sets(cands, run, device)
    owner.eager_tune_log = [(tuple(st.priority for st in sts), round(v * 1e3, 3)) for sts, v in zip(cands, score)]
    cache[key] = cands[k]
    return cands[k]


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

    def go(sts):
        for st in sts:
            x.record_stream(st)  # x may be freed by the caller while the side streams still read it
        fork_parts(sts, cur, [lambda i=i: part_fn(x[bounds[i]:bounds[i + 1]], i, out=logits[bounds[i]:bounds[i + 1]])
                              for i in range(ns)])

    owner._streams = part_streams(owner, (B, ns, str(dev), tuple(bounds)), ns, go, dev,
                                  getattr(owner, "stream_priorities", None))
    go(owner._streams)
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
    next call), as the eager forward does.

    A split forward (one that forks its batch parts through fork_parts) is captured as one graph per
    part, each replayed on its part stream (see fork_parts); other forwards as one graph."""

    def __init__(self, max_entries: int = 4):
        self.max_entries = max_entries
        self._entries = {}
        self.captures = 0
        self.tune_log = None

    def clear(self):
        self._entries = {}

    def _capture(self, key, x, forward, keep):
        if len(self._entries) >= self.max_entries:
            self._entries = {}
        dev = x.device
        cur = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(cur)
        _NO_TUNE[0] += 1
        try:
            with torch.cuda.stream(side):
                forward(x)  # first launches (kernel attributes), packing and workspaces outside the capture
        finally:
            _NO_TUNE[0] -= 1
        cur.wait_stream(side)
        torch.cuda.synchronize(dev)
        # a split forward (fork_parts) first: each part captured into a graph of its own on its own
        # stream, everything outside the parts (cached packing) run eagerly -- it queues no kernel on a
        # repeat call, so the part graphs are the whole forward
        parts = []
        _PART_CAPTURE[0] = parts if PART_GRAPHS[0] else None
        _NO_TUNE[0] += 1
        try:
            out = forward(x)
        finally:
            _PART_CAPTURE[0] = None
            _NO_TUNE[0] -= 1
        torch.cuda.synchronize(dev)
        if parts:
            g = self._tune(parts, dev)
        else:
            g = torch.cuda.CUDAGraph()
            # thread_local: HIP calls other threads make meanwhile (e.g. a process group's watchdog)
            # neither break this capture nor are broken by it.  A refused capture raises (measured:
            # after one, the next launch on the device fails too, so there is no eager fallback)
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                out = forward(x)
        self.captures += 1
        e = self._entries[key] = (g, out, x, (x,) + tuple(keep()))
        return e

    def _tune(self, parts, device):
        """The part graphs replayed on TUNE_CANDIDATES stream sets -- the capture's own, then fresh
        pick_streams sets, alternately all at priority 0 and part 0 at high priority -- after three warm-up
        replays, four timed replays each over two passes in opposite orders; the set with the lowest
        second-best time is kept ((priorities, ms) per set in tune_log).

        Why measured: whether two stream parts overlap depends on which streams they run on, through
        state no probe of this round predicted (round 6, tools/exp_vivit_hwq.py / ab_stream_modes.py:
        ViViT-B B = 8 850-900 vs 960-1000 clips/s, ResNet3D-50 990 vs 1517, TimeSformer-B 1430 vs 1829
        from one stream set to the next, every set stable over repeated replays in its process)."""
        n = len(parts)
        graphs = [pg for _, pg in parts]
        # (one candidate per assignment of the parts to distinct hardware queues instead, all at priority 0,
        # ran 953-963 clips/s where these sets gave 956-991 on the same box: profiles/r06_hwq.txt)
        cands = _candidate_sets(device, n, [st for st, _ in parts])
        k, score = _rank_sets(cands, lambda sts: self._replay(list(zip(sts, graphs)), device), device)
        self.tune_log = [(tuple(st.priority for st in sts), round(v * 1e3, 3)) for sts, v in zip(cands, score)]
        return list(zip(cands[k], graphs))

    @staticmethod
    def _replay(g, device):
        if isinstance(g, list):  # part graphs: each on its own stream, forked from and joined to the caller's
            cur = torch.cuda.current_stream(device)
            for st, pg in g:
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    pg.replay()
            for st, _ in g:
                cur.wait_stream(st)
        else:
            g.replay()

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
                self._replay(g, x.device)
                return out
            e = self._capture(key, x, forward, keep)
        g, out, _, _ = e
        self._replay(g, x.device)
        return out
