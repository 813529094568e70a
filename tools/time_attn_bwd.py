"""Time the attention forward (with LSE) and backward kernels at the ViViT-B train shape
(B clips x 12 heads x 3137 tokens, head_dim 64) with HIP events; prints TFLOP/s per launch."""
import sys
import time

import torch

sys.path.insert(0, ".")
from vclip_amd import ops  # noqa: E402

B, S, H = int(sys.argv[1]) if len(sys.argv) > 1 else 4, 3137, 12
rows = (B - 1) * S + (S + 63) // 64 * 64 + 128
g = torch.Generator(device="cuda").manual_seed(0)
qkv = (torch.randn(rows, 3 * H * 64, device="cuda", generator=g) * 0.5).bfloat16()
dout = (torch.randn(rows, H * 64, device="cuda", generator=g) * 0.1).bfloat16()
out = torch.zeros(rows, H * 64, device="cuda", dtype=torch.bfloat16)
lse = torch.zeros(B * H * S, device="cuda")
delta = torch.zeros_like(lse)
dqkv = torch.zeros_like(qkv)
gf = 4 * S * S * 64 * H * B / 1e9  # one QK^T + one PV
for name, fn, mult in (("fwd_lse", lambda: ops.attention_fwd_lse(qkv, B, S, H, out, lse), 1),
                       ("bwd", lambda: ops.attention_bwd(qkv, out, dout, lse, delta, B, S, H, dqkv), 2)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name}: {ms * 1e3:.1f} us  {gf * mult / ms:.1f} TFLOP/s (algorithmic)")
