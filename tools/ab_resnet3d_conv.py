"""Interleaved A/B of the ResNet3D-50 B = 4 headline (2 streams, graph replay) over per-convolution
(ring, tile) overrides (model.conv_cfg, vc_conv3d_gemm_bf16_cfg), one process; logits must be
bit-identical.  python tools/ab_resnet3d_conv.py '{}' '{"conv_a.s5": [4, 1], "conv_b.s5": [4, 1]}'"""
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
ap.add_argument("cfgs", nargs="+")
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
B = 4
x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
m = create_model(device=dev).eval()
m.graph_replay = True
m.concurrent_streams = 2
cfgs = [{k: tuple(v) for k, v in json.loads(c).items()} for c in a.cfgs]
outs = []
for c in cfgs:
    m.conv_cfg = c
    outs.append(m.forward_logits(x).clone())
print("logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in cfgs]
for r in range(a.rounds):
    for i in (range(len(cfgs)) if r % 2 == 0 else reversed(range(len(cfgs)))):
        m.conv_cfg = cfgs[i]
        for _ in range(2):
            m.forward_logits(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            m.forward_logits(x)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 20 * 1e3)
for c, t in zip(a.cfgs, res):
    print(f"resnet3d conv_cfg={c}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({B / np.median(t) * 1e3:.1f} clips/s)",
          flush=True)
