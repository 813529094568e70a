"""Data-parallel gradient exchange for the ViViT train step (BASELINE config 5:
"ViViT-B train step ... DP=8 grad all-reduce over xGMI").

The reference has no distributed code (one GPU, `cuda:1`, vivit_transformer/main.py:83).  The
build shards clips across ranks (one process per GPU, torch.distributed with the nccl backend =
RCCL over xGMI); the one real exchange is the gradient all-reduce before AdamW.  Gradients live
in one flat fp32 buffer whose layout puts layers in the order the backward finishes them
(vclip_amd.vivit_train.FlatLayout), so each finished stage is a contiguous slice: it is bucketed
(adjacent stages merged up to `bucket_bytes`) and all-reduced on a side stream while the
backward of the layers below keeps the compute stream busy.  `wait()` joins the side stream
before the optimizer step; the average (SUM then x 1/world) happens on the side stream too.

Usage (the reference loop plus two lines):
    sync = GradAllReduce(model)                  # after torch.distributed.init_process_group
    ...; loss.backward(); sync.wait(); optimizer.step()
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradAllReduce:
    def __init__(self, model, group=None, bucket_bytes: int = 32 << 20, average: bool = True):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.average = average
        self._pending = None  # (start, end, gflat) accumulated but not yet launched
        self._side = None
        self._launched = []  # (start, end) ranges, for tests
        model.grad_ready_hooks.append(self._on_ready)

    def _stream(self, device):
        if device.type != "cuda":
            return None
        if self._side is None:
            from . import streams  # the train step's third side stream (vivit_train: wgrad, dQ)
            self._side = streams.pick_streams(device, 3, against=(torch.cuda.current_stream(device),))[2]
        return self._side

    def _on_ready(self, stage, start, end, gflat):
        if self._pending is None:
            self._pending = [start, end, gflat]
        else:
            assert self._pending[1] == start and self._pending[2] is gflat, "stages must complete in flat order"
            self._pending[1] = end
        last = stage == "embeddings"
        if last or self._pending[1] - self._pending[0] >= self.bucket_elems:
            self._launch()

    def _launch(self):
        start, end, gflat = self._pending
        self._pending = None
        buf = gflat[start:end]
        side = self._stream(gflat.device)
        if side is None:  # CPU / gloo: synchronous
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            if self.average and self.world > 1:
                buf.mul_(1.0 / self.world)
        else:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(gflat.device))
            side.wait_event(ev)
            with torch.cuda.stream(side):
                # RCCL averages in the collective itself (ncclAvg); the work's wait() orders the
                # side stream after RCCL's internal stream without blocking the host
                op = dist.ReduceOp.AVG if self.average else dist.ReduceOp.SUM
                dist.all_reduce(buf, op=op, group=self.group, async_op=True).wait()
        self._launched.append((start, end))

    def wait(self):
        """Make the current stream wait for every launched all-reduce (call before optimizer.step())."""
        if self._pending is not None:
            self._launch()
        if self._side is not None:
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
        launched, self._launched = self._launched, []
        return launched
