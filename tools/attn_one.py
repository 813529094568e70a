"""Run the attention kernel N times (for rocprofv3 --pmc passes)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops
B, S, H = 8, 3137, 12
it = int(sys.argv[1]) if len(sys.argv) > 1 else 5
qkv = torch.randn(25344, 2304, device="cuda").bfloat16()
o = torch.zeros(25344, 768, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    ops.attention(qkv, B, S, H, 0.125, o)
torch.cuda.synchronize()
print("ok")
