"""Interleaved A/B of ViViT-B forward GEMM tile choices in one process (cdna_hip_programming.md §5.4
rule 24): python tools/ab_model_cfg.py '{}' '{"o_proj": 7, "fc2": 7}' [--B 8] [--streams 2] —
times model.forward_logits under each model.gemm_cfg in alternating rounds; logits must match.
A list value gives one config per stream part ({"fc1": [26, 25]}); the key "_rows" sets model.rows for
that variant ("pad" / "tight"), "_prio" the per-part HIP stream priorities ([-1, 0]: part 0 high), "_split"
the clips per part, "_streams" the number of parts."""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("cfgs", nargs="+")
ap.add_argument("--B", type=int, default=8)
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--rounds", type=int, default=8)
ap.add_argument("--graph", type=int, default=1, help="replay captured hipGraphs (the bench's default)")
ap.add_argument("--rows", default=None, help="model.rows ('tight': B*S rows rounded to the tile height)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
pix = torch.from_numpy(make_synthetic_clips(a.B, 32, 224, seed=1)).to(dev)
m = create_model(num_frames=32, device=dev)
m.concurrent_streams = a.streams
m.graph_replay = bool(a.graph)
if a.rows:
    m.rows = a.rows
cfgs = [json.loads(c) for c in a.cfgs]


def apply(c):
    c = dict(c)
    m.rows = c.pop("_rows", a.rows or "pad")
    m.stream_priorities = c.pop("_prio", None)
    m.split_sizes = c.pop("_split", None)
    m.concurrent_streams = c.pop("_streams", a.streams)
    m.gemm_cfg = c


outs = []
for c in cfgs:
    apply(c)
    outs.append(m.forward_logits(pix).clone())
print("logits identical:", [bool(torch.equal(o, outs[0])) for o in outs], flush=True)
res = [[] for _ in cfgs]
for r in range(a.rounds):
    for i in (range(len(cfgs)) if r % 2 == 0 else reversed(range(len(cfgs)))):
        apply(cfgs[i])
        for _ in range(2):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 10 * 1e3)
for c, t in zip(a.cfgs, res):
    print(f"gemm_cfg={c}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({a.B / np.median(t) * 1e3:.1f} clips/s)",
          flush=True)
