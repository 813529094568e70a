"""Interleaved A/B of the ResNet3D-50 inference forward (32x224^2, B clips): implicit-GEMM convolutions
(vc_conv3d_gemm_bf16) vs im2col + GEMM, in one process; logits must be bit-identical.
  python tools/ab_resnet3d.py [--B 4] [--streams 2] [--graph 1] [--rounds 6]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd.resnet3d import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_video  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4)
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--graph", type=int, default=1)
ap.add_argument("--rounds", type=int, default=6)
a = ap.parse_args()
dev = torch.device("cuda", 0)
x = torch.from_numpy(make_synthetic_video(a.B, 32, 224, seed=1)).to(dev)
m = create_model(device=dev).eval()
m.concurrent_streams = a.streams
m.graph_replay = bool(a.graph)
arms = {"implicit": True, "im2col": False}
outs = {}
for k, v in arms.items():
    m.implicit_conv = v
    outs[k] = m.forward_logits(x).clone()
print("logits max |diff|:", float((outs["implicit"] - outs["im2col"]).abs().max()), flush=True)
res = {k: [] for k in arms}
for r in range(a.rounds):
    for k in (list(arms) if r % 2 == 0 else list(reversed(list(arms)))):
        m.implicit_conv = arms[k]
        for _ in range(2):
            m.forward_logits(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(x)
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 10 * 1e3)
for k, t in res.items():
    print(f"{k}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({a.B / np.median(t) * 1e3:.1f} clips/s)",
          flush=True)
