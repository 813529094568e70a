"""Train-step throughput of the TimeSformer / Swin3D / ResNet3D families (each folder's loop:
zero_grad, forward, CrossEntropyLoss, backward, optimizer.step) on synthetic clips:
  python tools/time_train_families.py [timesformer swin resnet3d] [--steps 10]
One JSON line per family: clips/s, ms/step, the batch and the clip shape."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from vclip_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("families", nargs="*", default=["timesformer", "swin", "resnet3d"])
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--warmup", type=int, default=3)
a = ap.parse_args()
_lib.load()
dev = torch.device("cuda", 0)
from vclip_amd.optim import AdamW  # noqa: E402
from vclip_amd.weights import make_synthetic_clips, make_synthetic_video  # noqa: E402

for fam in a.families:
    if fam == "timesformer":
        from vclip_amd.timesformer import create_model
        B, shape = 8, "8x224^2"
        m = create_model(num_frames=8, device=dev).train()
        x = torch.from_numpy(make_synthetic_clips(B, 8, 224, seed=1)).to(dev)
        fwd = lambda: m(pixel_values=x).logits  # noqa: E731
        opt = AdamW(m.parameters(), lr=1e-5, weight_decay=0.01)
    elif fam == "swin":
        from vclip_amd.swin3d import create_model
        B, shape = 4, "32x224^2"
        m = create_model(model_size="tiny", device=dev).train()
        x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
        fwd = lambda: m(x)  # noqa: E731
        opt = AdamW(m.parameters(), lr=1e-4, weight_decay=0.05)
    else:
        from vclip_amd.resnet3d import create_model
        B, shape = 4, "32x224^2"
        m = create_model(device=dev).train()
        x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
        fwd = lambda: m(x)  # noqa: E731
        opt = AdamW([q for q in m.parameters() if q.requires_grad], lr=1e-3, weight_decay=0.0)
    y = torch.randint(0, 2, (B,), device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad()
        loss = crit(fwd(), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"family": fam, "mode": "train", "clips_per_s": round(B / dt, 2), "ms_per_step": round(dt * 1e3, 2),
                      "batch": B, "clip": shape, "loss": round(float(loss), 4)}), flush=True)
    del m, opt, x
    torch.cuda.empty_cache()
