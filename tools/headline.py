"""The bench headline alone (kernel traces and PMC passes of the timed configuration): the model
forward of `bench.py --mode M` over --streams HIP streams with graph replay, nothing else (no fp16
legs, no one-stream passes, no CPU oracle), so a rocprofv3 session of this command holds exactly the
kernels the headline times.

  python tools/headline.py [--mode fwd|timesformer|swin|resnet3d] [--streams 2] [--graph 1] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="fwd")
ap.add_argument("--streams", type=int, default=None)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--graph", type=int, default=1)
ap.add_argument("--batch", type=int, default=None)
ap.add_argument("--serial", type=int, default=0,
                help="1: the split's parts one after the other on one stream, eager (bench.py's roofline and "
                     "per-kernel passes: the same launches without the overlap)")
ap.add_argument("--gemm-cfg", default=None, help="JSON {op: cfg} override (ViViT: model.gemm_cfg)")
ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp16", "fp16_precise"),
                help="ViViT operand type: bench.py's fp16 / fp16_precise legs (compute_dtype, precise_layers = 1)")
ap.add_argument("--precise-ops", default=None, help="fp16_precise: comma list of split-operand GEMMs (model.precise_ops: embed|embed_w,qkv,o_proj,fc1,fc2)")
a = ap.parse_args()
if a.streams is None:
    a.streams = 4 if a.mode == "swin" else 2
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
if a.gemm_cfg:
    m.gemm_cfg = json.loads(a.gemm_cfg)
if a.dtype != "bf16":
    m.compute_dtype = torch.float16
    m.precise_layers = 1 if a.dtype == "fp16_precise" else 0
    if a.precise_ops:
        m.precise_ops = tuple(a.precise_ops.split(","))
m.concurrent_streams = a.streams
m.graph_replay = bool(a.graph) and not a.serial
from vclip_amd import streams  # noqa: E402
with streams.serial_parts(bool(a.serial)):
    for _ in range(a.warmup):
        m.forward_logits(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        m.forward_logits(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
print(json.dumps({"mode": a.mode, "dtype": a.dtype, "streams": a.streams, "graph": int(m.graph_replay), "serial": a.serial, "batch": x.shape[0],
                  "ms_per_step": round(dt * 1e3, 3), "clips_s": round(x.shape[0] / dt, 2)}), flush=True)
