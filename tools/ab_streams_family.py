"""Interleaved A/B of a family's inference forward over the number of concurrent HIP streams the
batch is split into (model.concurrent_streams, graph replay as in bench.py), in one process; logits
must be bit-identical.
  python tools/ab_streams_family.py resnet3d 2 4 [--B 4] [--rounds 8]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("family", choices=["resnet3d", "timesformer", "swin"])
ap.add_argument("streams", nargs="+", type=int)
ap.add_argument("--B", type=int, default=None)
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
if a.family == "resnet3d":
    from vclip_amd.resnet3d import create_model
    from vclip_amd.weights import make_synthetic_video
    B = a.B or 4
    x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
    m = create_model(device=dev).eval()
    fwd = lambda: m.forward_logits(x)  # noqa: E731
elif a.family == "swin":
    from vclip_amd.swin3d import create_model
    from vclip_amd.weights import make_synthetic_video
    B = a.B or 4
    x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
    m = create_model(device=dev).eval()
    fwd = lambda: m.forward_logits(x)  # noqa: E731
else:
    from vclip_amd.timesformer import create_model
    from vclip_amd.weights import make_synthetic_clips
    B = a.B or 16
    x = torch.from_numpy(make_synthetic_clips(B, 8, 224, seed=1)).to(dev)
    m = create_model(device=dev).eval()
    fwd = lambda: m.forward_logits(x)  # noqa: E731
m.graph_replay = True
outs = []
for s in a.streams:
    m.concurrent_streams = s
    outs.append(fwd().clone())
print("logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in a.streams]
for r in range(a.rounds):
    for i in (range(len(a.streams)) if r % 2 == 0 else reversed(range(len(a.streams)))):
        m.concurrent_streams = a.streams[i]
        for _ in range(2):
            fwd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fwd()
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 10 * 1e3)
for s, t in zip(a.streams, res):
    print(f"{a.family} streams={s}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({B / np.median(t) * 1e3:.1f} clips/s)",
          flush=True)
