"""Interleaved A/B of the ViViT-B train step (32x224^2, B clips, the reference loop with vclip AdamW)
over TrainEngine settings, in one process; default arms: weight / bias gradients on a side stream
(side_wgrad) vs one stream.
  python tools/ab_train_side.py ['{"side_wgrad": false}' '{"side_wgrad": true, "wgrad_max_splits": 4}' ...]
  (arm key "_chain_priority": -1 runs the step, i.e. the data-gradient chain, on a high-priority HIP stream, so the
  side streams' weight gradients yield to it)
                                    [--B 4] [--rounds 6] [--steps 5]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd.optim import AdamW  # noqa: E402
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("arms", nargs="*", default=['{"side_wgrad": false}', '{"side_wgrad": true}'])
ap.add_argument("--B", type=int, default=4)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda", 0)
model = create_model(num_frames=32, device=dev).train()
opt = AdamW(model.parameters(), lr=1e-3, weight_decay=0.01)
pix = torch.from_numpy(make_synthetic_clips(a.B, 32, 224, seed=1)).to(dev)
labels = torch.from_numpy(np.random.RandomState(2).randint(0, 2, size=a.B)).long().to(dev)
crit = torch.nn.CrossEntropyLoss()


def step():
    opt.zero_grad()
    loss = crit(model(pixel_values=pix).logits, labels)
    loss.backward()
    opt.step()


step()
eng = model._engine
arms = [json.loads(x) for x in a.arms]
hp = torch.cuda.Stream(device=dev, priority=-1)
print("stream priority range", torch.cuda.Stream.priority_range(), "hp", hp.priority, flush=True)


def run(arm):
    if arm.get("_chain_priority", 0) < 0:
        hp.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(hp):
            step()
        torch.cuda.current_stream(dev).wait_stream(hp)
    else:
        step()

res = [[] for _ in arms]
for r in range(a.rounds):
    for i in (range(len(arms)) if r % 2 == 0 else reversed(range(len(arms)))):
        for k, v in arms[i].items():
            if not k.startswith("_"):
                setattr(eng, k, v)
        run(arms[i])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            run(arms[i])
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / a.steps * 1e3)
for arm, t in zip(a.arms, res):
    print(f"{arm}: median {np.median(t):.3f} ms/step  min {min(t):.3f}  ({a.B / np.median(t) * 1e3:.1f} clips/s)",
          flush=True)
