"""The bench headline alone (for kernel traces): ViViT-B B=8 (or --mode family), --streams, graph replay."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="fwd")
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--graph", type=int, default=1)
ap.add_argument("--batch", type=int, default=None)
a = ap.parse_args()
from vclip_amd.weights import make_synthetic_clips, make_synthetic_video  # noqa: E402
if a.mode == "fwd":
    from vclip_amd.vivit import create_model
    m = create_model(num_frames=32, device="cuda")
    x = torch.from_numpy(make_synthetic_clips(a.batch or 8, 32, 224, seed=1)).cuda()
elif a.mode == "timesformer":
    from vclip_amd.timesformer import create_model
    m = create_model(num_frames=8, device="cuda")
    x = torch.from_numpy(make_synthetic_clips(a.batch or 16, 8, 224, seed=1)).cuda()
elif a.mode == "swin":
    from vclip_amd.swin3d import create_model
    m = create_model(model_size="tiny", device="cuda")
    x = torch.from_numpy(make_synthetic_video(a.batch or 4, 32, 224, seed=1)).cuda()
else:
    from vclip_amd.resnet3d import create_model
    m = create_model(device="cuda").eval()
    x = torch.from_numpy(make_synthetic_video(a.batch or 4, 32, 224, seed=1)).cuda()
m.concurrent_streams = a.streams
m.graph_replay = bool(a.graph)
for _ in range(3):
    m.forward_logits(x)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    m.forward_logits(x)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.steps
print(f"{a.mode} streams {a.streams} graph {a.graph}: {dt * 1e3:.3f} ms/step, {x.shape[0] / dt:.1f} clips/s", flush=True)
