"""Per-launch time and rate of the Swin-T window-attention kernel by stage (B=4, 32x224^2)."""
import sys

import torch

sys.path.insert(0, ".")
if len(sys.argv) > 2:  # optional A/B build: python tools/swin_attn_stages.py B path/to/libvclip.so
    from vclip_amd import _lib
    _lib.load(sys.argv[2])
from vclip_amd.swin3d import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_video  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
m = create_model(model_size="tiny", device=dev)
x = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
for _ in range(3):
    m.forward_logits(x)
torch.cuda.synchronize()
ev = []
m.kernel_events = ev
for _ in range(10):
    m.forward_logits(x)
torch.cuda.synchronize()
m.kernel_events = None
per = len(ev) // 10
for i in range(per):
    ts = [ev[k * per + i][0].elapsed_time(ev[k * per + i][1]) for k in range(10)]
    ts.sort()
    f = ev[i][2]
    tot = tot + ts[5] if i else ts[5]
    print(f"launch {i:2d}: {ts[5] * 1e3:7.1f} us  {f / 1e9:6.2f} GF  {f / (ts[5] * 1e-3) / 1e12:6.1f} TF/s", flush=True)
print(f"total {tot * 1e3:.1f} us per forward", flush=True)
