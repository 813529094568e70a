"""Logit error and speed of the ViViT-B operand-precision variants on the bench's 8 clips (one process):
bf16, fp16, and fp16 with split-operand GEMMs (model.precise_ops sets), each against the fp32 oracle run
on the GPU in fp32 (test infrastructure: the oracle is the checker, never the thing timed), and timed as
the headline runs (2 HIP streams, 5 + 3 clips, graph replay), alternating with bf16 re-runs.
  python tools/precision_legs.py [--rounds 6]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.vivit_ref import vivit_forward  # noqa: E402
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips, make_vivit_weights  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=6)
a = ap.parse_args()
dev = torch.device("cuda", 0)
m = create_model(num_frames=32, device=dev)
cfg = dict(m.config.as_shape_cfg(), num_attention_heads=m.config.num_attention_heads,
           layer_norm_eps=m.config.layer_norm_eps)
pix_np = make_synthetic_clips(8, 32, 224, seed=1)
pix = torch.from_numpy(pix_np).to(dev)
sd = make_vivit_weights(cfg, seed=0)
with torch.no_grad():
    ref = vivit_forward({k: torch.from_numpy(v).to(dev) for k, v in sd.items()}, cfg, pix).cpu().numpy()
m.concurrent_streams = 2
m.graph_replay = True
VARIANTS = [("bf16", torch.bfloat16, 0, ()), ("fp16", torch.float16, 0, ()),
            ("fp16+embed_w", torch.float16, 1, ("embed_w",)), ("fp16+embed_w+qkv", torch.float16, 1, ("embed_w", "qkv")),
            ("fp16+embed", torch.float16, 1, ("embed",))]


def setv(v):
    _, dt, pl, ops = v
    m.compute_dtype, m.precise_layers = dt, pl
    if ops:
        m.precise_ops = ops


errs = {}
for v in VARIANTS:
    setv(v)
    errs[v[0]] = float(np.abs(m.forward_logits(pix).cpu().numpy() - ref).max())
    print(f"{v[0]}: logit max|err| {errs[v[0]]:.3e}", flush=True)
times = {v[0]: [] for v in VARIANTS}
base = {v[0]: [] for v in VARIANTS}


def timeit(n=10):
    for _ in range(2):
        m.forward_logits(pix)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        m.forward_logits(pix)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for r in range(a.rounds):
    for v in (VARIANTS if r % 2 == 0 else VARIANTS[::-1]):
        setv(v)
        times[v[0]].append(timeit())
        setv(VARIANTS[0])
        base[v[0]].append(timeit())
for v in VARIANTS:
    t, tb = np.median(times[v[0]]), np.median(base[v[0]])
    print(f"{v[0]:>18}: {8 / t * 1e3:7.1f} clips/s ({t:.3f} ms), bf16 beside it {8 / tb * 1e3:7.1f}: "
          f"ratio {tb / t:.4f}; logit err {errs[v[0]]:.3e}", flush=True)
