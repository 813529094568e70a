"""Interleaved A/B of the ResNet3D-50 inference forward (32x224^2, B clips) over implicit-conv LDS
ring depths per res stage (model.conv_ring, vc_conv3d_gemm_bf16_ring), in one process; logits must be
bit-identical.
  python tools/ab_resnet3d_ring.py '{}' '{"s5": 3}' '{"s4": 3, "s5": 3}' [--B 4] [--rounds 8]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd.resnet3d import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_video  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("arms", nargs="+")
ap.add_argument("--B", type=int, default=4)
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--graph", type=int, default=1)
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
x = torch.from_numpy(make_synthetic_video(a.B, 32, 224, seed=1)).to(dev)
m = create_model(device=dev).eval()
m.concurrent_streams = a.streams
m.graph_replay = bool(a.graph)
arms = [json.loads(s) for s in a.arms]
outs = []
for arm in arms:
    m.conv_ring = arm
    outs.append(m.forward_logits(x).clone())
print("logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in arms]
for r in range(a.rounds):
    for i in (range(len(arms)) if r % 2 == 0 else reversed(range(len(arms)))):
        m.conv_ring = arms[i]
        for _ in range(2):
            m.forward_logits(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(x)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 10 * 1e3)
for arm, t in zip(a.arms, res):
    print(f"conv_ring={arm}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({a.B / np.median(t) * 1e3:.1f} clips/s)",
          flush=True)
