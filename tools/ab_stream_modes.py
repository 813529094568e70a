"""Interleaved A/B of how a split forward's parts are issued (one process, graph replay, logits must match):
part graphs on the stream set GraphReplay._tune timed fastest, part graphs on the picked streams
(default priorities / all 0), and one graph holding every branch (streams.PART_GRAPHS).
  python tools/ab_stream_modes.py <vivit|swin|resnet3d|timesformer> [--rounds 4]"""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd import streams  # noqa: E402
from vclip_amd.weights import make_synthetic_clips, make_synthetic_video  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("family")
ap.add_argument("--rounds", type=int, default=4)
a = ap.parse_args()
dev = torch.device("cuda", 0)
if a.family == "vivit":
    from vclip_amd.vivit import create_model
    m, B, ns = create_model(num_frames=32, device=dev), 8, 2
    x = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
elif a.family == "timesformer":
    from vclip_amd.timesformer import create_model
    m, B, ns = create_model(num_frames=8, device=dev), 16, 2
    x = torch.from_numpy(make_synthetic_clips(B, 8, 224, seed=1)).to(dev)
elif a.family == "swin":
    from vclip_amd.swin3d import create_model
    m, B, ns = create_model(model_size="tiny", device=dev), 4, 4
    x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
else:
    from vclip_amd.resnet3d import create_model
    m, B, ns = create_model(device=dev), 4, 2
    x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
m.concurrent_streams = ns
zeros = (0,) * ns
modes = [("part graphs, tuned", True, None, 6), ("part graphs, prio -1 0..", True, (-1,) + zeros[1:], 1),
         ("part graphs, prio 0", True, zeros, 1), ("one graph, prio 0", False, zeros, 1)]


def apply(mode):
    _, pg, pr, tc = mode
    streams.PART_GRAPHS[0] = pg
    streams.TUNE_CANDIDATES[0] = tc
    m.stream_priorities = pr
    if m._graphs is not None:
        m._graphs.clear()
    m.graph_replay = True


outs = []
for md in modes:
    apply(md)
    outs.append(m.forward_logits(x).clone())
print(a.family, "logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in modes]
for r in range(a.rounds):
    for i in (range(len(modes)) if r % 2 == 0 else reversed(range(len(modes)))):
        apply(modes[i])
        for _ in range(3):
            m.forward_logits(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(x)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 10 * 1e3)
for md, t in zip(modes, res):
    print(f"  {md[0]:28s} median {np.median(t):.3f} ms  ({B / np.median(t) * 1e3:.1f} clips/s)  "
          f"rounds {' '.join(f'{v:.2f}' for v in t)}", flush=True)
print("  picks concurrent:", streams.PICK_STATUS, flush=True)
apply(modes[0])
m.forward_logits(x)
print("  last tuning (priorities, ms):", m._graphs.tune_log, flush=True)
