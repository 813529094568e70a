"""Forward (or train-step) time of one libvclip.so build, for process-level A/B of two builds
on the same box (tools/ab_build.sh makes ab/<name>/libvclip.so from a git revision):
  python tools/ab_lib.py <path/to/libvclip.so> [fwd|train|timesformer|swin|resnet3d] [steps]
The library is bound before any op runs, so every kernel of the run comes from it."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd import _lib  # noqa: E402

path, mode = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "fwd")
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
_lib.load(path)
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

dev = torch.device("cuda", 0)
B = {"fwd": 8, "timesformer": 16}.get(mode, 4)
if mode == "timesformer":
    from vclip_amd.timesformer import create_model as tsf_model
    m = tsf_model(num_frames=8, device=dev)
    pix = torch.from_numpy(make_synthetic_clips(B, 8, 224, seed=1)).to(dev)
elif mode == "swin":
    from vclip_amd.swin3d import create_model as swin_model
    from vclip_amd.weights import make_synthetic_video
    m = swin_model(model_size="tiny", device=dev)
    pix = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
elif mode == "resnet3d":
    from vclip_amd.resnet3d import create_model as r3d_model
    from vclip_amd.weights import make_synthetic_video
    m = r3d_model(device=dev)
    pix = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
else:
    m = create_model(num_frames=32, device=dev)
    pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
if mode != "train":
    # the bench's headline configuration: the batch over its HIP streams, replayed from a captured hipGraph
    m.concurrent_streams = 4 if mode == "swin" else 2
    m.graph_replay = True
    step = lambda: m.forward_logits(pix)  # noqa: E731
else:
    from vclip_amd.optim import AdamW
    m.train()
    opt = AdamW(m.parameters(), lr=1e-3, weight_decay=0.01)
    y = torch.from_numpy(np.random.RandomState(2).randint(0, 2, size=B)).long().to(dev)

    def step():
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(pixel_values=pix).logits, y).backward()
        opt.step()
for _ in range(5):
    step()
torch.cuda.synchronize()
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    for _ in range(steps // 3):
        step()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) / (steps // 3) * 1e3)
extra = ""
if mode in ("swin", "fwd", "timesformer") and hasattr(m, "kernel_events"):
    # mean attention launch (HIP events on the launching stream; one stream, eager)
    m.concurrent_streams = 1
    m.graph_replay = False
    evs = []
    m.kernel_events = evs
    for _ in range(3):
        step()
    m.kernel_events = None
    torch.cuda.synchronize()
    extra = f", attention {np.mean([e[0].elapsed_time(e[1]) for e in evs]) * 1e3:.1f} us/launch"
from vclip_amd import streams  # noqa: E402
print(f"{path} {mode}: {min(ts):.3f} ms/step (min of 3), {B / min(ts) * 1e3:.1f} clips/s{extra}"
      f"  picked streams concurrent {streams.PICK_STATUS}", flush=True)
