"""ViViT-B B=8 forward with the batch on 1 vs 2 concurrent HIP streams (interleaved rounds, one process):
clips/s, and the per-op HIP-event launch time in each mode (events on the stream each launch runs on)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

dev = torch.device("cuda", 0)
B = 8
pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
m = create_model(num_frames=32, device=dev)
res = {1: [], 2: []}
for rnd in range(4):
    for ns in (1, 2):
        m.concurrent_streams = ns
        for _ in range(3):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(15):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        res[ns].append(B * 15 / (time.perf_counter() - t0))
print({ns: f"median {np.median(v):.1f} max {max(v):.1f} clips/s" for ns, v in res.items()}, flush=True)
for ns in (1, 2):
    m.concurrent_streams = ns
    ev = {}
    m.kernel_events = ev
    for _ in range(5):
        m.forward_logits(pix)
    torch.cuda.synchronize()
    m.kernel_events = None
    print(ns, {k: round(float(np.mean([a.elapsed_time(b) for a, b in v])) * 1000, 1) for k, v in ev.items()}, flush=True)
