"""ViViT-B B = 4 train step (eager) on several side-stream sets: the weight-gradient side stream and the
attention backward's dQ stream re-drawn from torch's pool per trial (k dummy streams first), half the
trials from streams.pick_streams (pairwise on different hardware queues, measured).  Does the train
step have the forward's two-stream lottery (profiles/r06_hwq.txt)?
  python tools/exp_train_streams.py [--trials 8]"""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd import ops, streams  # noqa: E402
from vclip_amd.optim import AdamW  # noqa: E402
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--trials", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
B = 4
m = create_model(num_frames=32, device=dev)
m.train()
opt = AdamW(m.parameters(), lr=1e-3, weight_decay=0.01)
pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
y = torch.from_numpy(np.random.RandomState(2).randint(0, 2, size=B)).long().to(dev)


def step():
    opt.zero_grad()
    torch.nn.functional.cross_entropy(m(pixel_values=pix).logits, y).backward()
    opt.step()


NB = 4 * 32 * torch.cuda.get_device_properties(dev).multi_processor_count


def behind(x, z, iters=24):
    """one-workgroup spin on z behind a four-round spin on x: z's completion over x's (tools/hwq_pipe_probe.py)"""
    best = 9.0
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(x):
            ops.spin(iters, dev, NB)
        with torch.cuda.stream(z):
            ops.spin(1, dev, 1)
        z.synchronize()
        tb = time.perf_counter() - t0
        x.synchronize()
        best = min(best, tb / (time.perf_counter() - t0))
    return best


def timeit():
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 8


for _ in range(3):
    step()
for k in range(a.trials):
    for _ in range(k):
        torch.cuda.Stream(device=dev)
    eng = m._engine
    if k % 2:
        eng.side, eng.side_dq = streams.pick_streams(dev, 2, fresh=True)
        how = "picked (fresh)"
    elif k == 0:
        how = f"default (the engine's own picks, ok {list(streams.PICK_STATUS.values())})"
    else:
        eng.side, eng.side_dq = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
        how = "pool"
    t = timeit()
    main = torch.cuda.current_stream(dev)
    pr = {nm: f"{behind(x, z):.2f}/{behind(z, x):.2f}" for nm, (x, z) in
          (("main-side", (main, eng.side)), ("main-dq", (main, eng.side_dq)), ("side-dq", (eng.side, eng.side_dq)))}
    print(f"k={k} {how}: {t * 1e3:.2f} ms/step ({B / t:.1f} clips/s)  dispatch probe {pr}", flush=True)
