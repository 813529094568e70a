"""ViViT-B B = 4 train step: the eager step vs GraphedTrainStep captured several times in one process (every
capture a new instantiation, whose branch streams HIP chooses; profiles/r06_hwq.txt).  Timing only: the
replays are real optimizer steps.
  python tools/exp_train_graph.py [--captures 4]"""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd.optim import AdamW  # noqa: E402
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.vivit_train import GraphedTrainStep  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--captures", type=int, default=4)
a = ap.parse_args()
dev = torch.device("cuda", 0)
B = 4
m = create_model(num_frames=32, device=dev)
m.train()
opt = AdamW(m.parameters(), lr=1e-5, weight_decay=0.01)
crit = torch.nn.CrossEntropyLoss()
pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
y = torch.from_numpy(np.random.RandomState(2).randint(0, 2, size=B)).long().to(dev)


def eager():
    opt.zero_grad()
    crit(m(pixel_values=pix).logits, y).backward()
    opt.step()


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return B * n / (time.perf_counter() - t0)


print(f"eager: {timeit(eager):.1f} clips/s", flush=True)
for c in range(a.captures):
    g = GraphedTrainStep(m, opt, crit, pix, y)
    print(f"capture {c}: {timeit(lambda: g(pix, y)):.1f} clips/s   eager again {timeit(eager):.1f}", flush=True)
    del g
