"""Time the short-sequence attention (S <= 256) at TimeSformer-B's spatial geometry: B*T = 16*8
sequences of 197 tokens, 12 heads, q|k|v rows of 2304 (the fused projection output).  Prints
the mean launch time over `iters` launches (HIP events), the algorithmic HBM rate (q, k, v read
once, out written once) and the MFMA rate.  The kernel variant comes from VC_ATTN_SHORT_VARIANT
(read once per process).  Usage: python tools/time_short_attn.py [iters] [sequences]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 50
B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
S, H = 197, 12
rows = B * S + 64
qkv = torch.randn(rows, 3 * H * 64, device="cuda").bfloat16()
o = torch.zeros(rows, H * 64, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    ops.attention(qkv, B, S, H, 0.125, o, q_prescaled=True)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    ops.attention(qkv, B, S, H, 0.125, o, q_prescaled=True)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / it * 1e3
byts = B * H * S * 64 * 2 * 4
flop = 4.0 * B * H * S * S * 64
print(json.dumps({"variant": os.environ.get("VC_ATTN_SHORT_VARIANT", "default"), "sequences": B, "us": round(us, 2),
                  "GB/s": round(byts / us * 1e-3, 1), "hbm_frac": round(byts / us * 1e-3 / 8000, 4),
                  "TFLOP/s": round(flop / us * 1e-6, 1), "mfma_frac": round(flop / us * 1e-6 / 2500, 4)}))
