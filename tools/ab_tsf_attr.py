"""Interleaved A/B of a TimeSformer-B forward attribute in one process (cdna_hip_programming.md §5.4
rule 24): python tools/ab_tsf_attr.py <attr> <json value A> <json value B> [--B 16] [--streams 2] —
model.forward_logits timed with the attribute at each value in alternating rounds; logits compared."""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd.timesformer import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("attr")
ap.add_argument("values", nargs="+")
ap.add_argument("--B", type=int, default=16)
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
x = torch.from_numpy(make_synthetic_clips(a.B, 8, 224, seed=1)).to(dev)
m = create_model(num_frames=8, device=dev)
m.concurrent_streams = a.streams
vals = [json.loads(v) for v in a.values]
outs = []
for v in vals:
    setattr(m, a.attr, v)
    outs.append(m.forward_logits(x).clone())
print("logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in vals]
for r in range(a.rounds):
    for i in (range(len(vals)) if r % 2 == 0 else reversed(range(len(vals)))):
        setattr(m, a.attr, vals[i])
        for _ in range(2):
            m.forward_logits(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(x)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 10 * 1e3)
for v, t in zip(a.values, res):
    print(f"{a.attr}={v}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({a.B / np.median(t) * 1e3:.1f} clips/s)",
          flush=True)
