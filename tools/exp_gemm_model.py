"""ViViT-B B=8 forward on two HIP streams (the bench's headline mode), one process, interleaved rounds:
vc_gemm's own tile pick vs each alternative config of ONE projection GEMM at a time (model.gemm_cfg),
with padded or tight row counts (model.rows).  Prints clips/s (median of rounds) per variant."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

dev = torch.device("cuda", 0)
B = 8
streams = int(sys.argv[1]) if len(sys.argv) > 1 else 2
pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
m = create_model(num_frames=32, device=dev)
m.concurrent_streams = streams
variants = [("auto/pad", {}, "pad"), ("auto/tight", {}, "tight")]
for name, cfgs in (("qkv", (3, 5, 0)), ("o_proj", (3, 0, 2, 7)), ("fc1", (3, 5)), ("fc2", (5, 0, 2))):
    for c in cfgs:
        variants.append((f"{name}={c}/pad", {name: c}, "pad"))
ref = m.forward_logits(pix).clone()
ok = []
for label, gc, rows in variants:
    m.gemm_cfg, m.rows = gc, rows
    try:
        lg = m.forward_logits(pix).clone()
        torch.cuda.synchronize()
    except Exception as e:  # a config that does not tile this shape
        print(f"{label}: skipped ({e})", flush=True)
        continue
    d = (lg - ref).abs().max().item()
    print(f"{label}: logits max |diff| vs auto/pad {d:.3e}", flush=True)
    ok.append((label, gc, rows))
res = {v[0]: [] for v in ok}
for rnd in range(5):
    for label, gc, rows in ok:
        m.gemm_cfg, m.rows = gc, rows
        for _ in range(2):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(12):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        res[label].append(B * 12 / (time.perf_counter() - t0))
for label, v in res.items():
    print(f"{label:16s} median {np.median(v):7.1f}  max {max(v):7.1f} clips/s", flush=True)
