"""Interleaved A/B of a ViViT-B forward switch in one process (cdna_hip_programming.md §5.4
rule 24): python tools/ab_model.py <attr> [B] — times model.forward_logits with the model
attribute <attr> False / True in alternating rounds and checks the logits are bit-identical."""
import sys
import time

import torch

sys.path.insert(0, ".")
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

attr = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dev = torch.device("cuda", 0)
pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
m = create_model(num_frames=32, device=dev)
outs = {}
for v in (False, True):
    setattr(m, attr, v)
    outs[v] = m.forward_logits(pix).clone()
print("bit-identical:", bool(torch.equal(outs[False], outs[True])), flush=True)
res = {False: [], True: []}
for rnd in range(6):
    for v in (False, True):
        setattr(m, attr, v)
        for _ in range(2):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / 10 * 1e3)
for v, ts in res.items():
    ts.sort()
    print(f"{attr}={v}: median {ts[len(ts) // 2]:.3f} ms/step  min {ts[0]:.3f}  ({B / ts[len(ts) // 2] * 1e3:.1f} clips/s)", flush=True)
