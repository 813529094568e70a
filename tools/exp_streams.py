"""ViViT-B B=8 forward: the batch on 1 HIP stream vs n streams (model.concurrent_streams), interleaved
rounds in one process, every round's clips/s printed (the spread matters).  Round-3 measurements of
the schedules not shipped (layer-by-layer round-robin enqueue, attention launches chained across the
streams, part i+1 started at a fixed op of part i's first layer) are recorded in DESIGN.md."""
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
VAR = [1, 2, 3]
ref = m.forward_logits(pix).clone()
for ns in VAR:
    m.concurrent_streams = ns
    assert torch.equal(m.forward_logits(pix), ref), ns
res = {v: [] for v in VAR}
for rnd in range(8):
    for v in VAR:
        m.concurrent_streams = v
        for _ in range(2):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(12):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        res[v].append(B * 12 / (time.perf_counter() - t0))
for v, x in res.items():
    print(f"streams {v}: median {np.median(x):.1f} min {min(x):.1f} max {max(x):.1f}  "
          f"{[round(u) for u in x]}", flush=True)
