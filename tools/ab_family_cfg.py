"""Interleaved A/B of a family's inference forward over per-GEMM tile overrides (model.gemm_cfg), graph
replay and the bench's stream count, in one process; logits must be bit-identical (every tile config
runs the same MFMA chain per output).
  python tools/ab_family_cfg.py timesformer '{}' '{"fc1": 8}' [--B 16] [--rounds 8]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("family", choices=["timesformer", "vivit"])
ap.add_argument("cfgs", nargs="+")
ap.add_argument("--B", type=int, default=None)
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

if a.family == "timesformer":
    from vclip_amd.timesformer import create_model
    B = a.B or 16
    x = torch.from_numpy(make_synthetic_clips(B, 8, 224, seed=1)).to(dev)
else:
    from vclip_amd.vivit import create_model
    B = a.B or 8
    x = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
m = create_model(device=dev).eval()
m.graph_replay = True
m.concurrent_streams = a.streams
cfgs = [json.loads(c) for c in a.cfgs]
outs = []
for c in cfgs:
    m.gemm_cfg = c
    outs.append(m.forward_logits(x).clone())
print("logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in cfgs]
for r in range(a.rounds):
    for i in (range(len(cfgs)) if r % 2 == 0 else reversed(range(len(cfgs)))):
        m.gemm_cfg = cfgs[i]
        for _ in range(2):
            m.forward_logits(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(x)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 10 * 1e3)
for c, t in zip(cfgs, res):
    print(f"{a.family} gemm_cfg={json.dumps(c)}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  "
          f"({B / np.median(t) * 1e3:.1f} clips/s)", flush=True)
