"""Interleaved A/B of a family's headline over the clips per stream part (model.split_sizes), graph
replay, one process; logits must be bit-identical (batch-invariant kernels).
  python tools/ab_split_sizes.py 4,4 5,3 6,2 3,3,2 [--family vivit|timesformer|resnet3d|swin]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd.weights import make_synthetic_clips, make_synthetic_video  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("splits", nargs="+")
ap.add_argument("--rounds", type=int, default=8)
ap.add_argument("--family", default="vivit", choices=["vivit", "timesformer", "resnet3d", "swin"])
a = ap.parse_args()
dev = torch.device("cuda", 0)
splits = [[int(v) for v in s.split(",")] for s in a.splits]
B = sum(splits[0])
if a.family == "vivit":
    from vclip_amd.vivit import create_model
    x = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
    m = create_model(num_frames=32, device=dev)
elif a.family == "timesformer":
    from vclip_amd.timesformer import create_model
    x = torch.from_numpy(make_synthetic_clips(B, 8, 224, seed=1)).to(dev)
    m = create_model(device=dev).eval()
else:
    create_model = __import__(f"vclip_amd.{'resnet3d' if a.family == 'resnet3d' else 'swin3d'}",
                              fromlist=["create_model"]).create_model
    x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
    m = create_model(device=dev).eval()
m.graph_replay = True


def use(sp):
    m.concurrent_streams = len(sp)
    m.split_sizes = sp


outs = []
for sp in splits:
    use(sp)
    outs.append(m.forward_logits(x).clone())
print("logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in splits]
for r in range(a.rounds):
    for i in (range(len(splits)) if r % 2 == 0 else reversed(range(len(splits)))):
        use(splits[i])
        for _ in range(2):
            m.forward_logits(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(x)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 10 * 1e3)
for sp, t in zip(splits, res):
    print(f"{a.family} split {sp}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({B / np.median(t) * 1e3:.1f} clips/s)", flush=True)
