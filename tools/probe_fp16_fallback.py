"""How often does the fp16 attention repeat its pass?  Per ViViT-B layer (fp16-operand forward, one
clip): the scores q'.k (log2 units; the scale is folded into q), each query row's max over all keys
minus its max over tile 0 (keys 0-63; the inference kernel's base).  fp16 P = exp2(s - m0) overflows
above 2^16, so a 128-query workgroup with any row past 16 (or a row sum past 65504) repeats its
pass with per-tile re-basing.  Prints, per layer, the share of rows and of workgroups affected.
  python tools/probe_fp16_fallback.py [--dtype fp16|bf16]"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from vclip_amd import ops  # noqa: E402
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="fp16")
a = ap.parse_args()
dev = torch.device("cuda", 0)
m = create_model(num_frames=32, device=dev)
m.compute_dtype = torch.float16 if a.dtype == "fp16" else torch.bfloat16
pix = torch.from_numpy(make_synthetic_clips(1, 32, 224, seed=1)).to(dev)
real = ops.attention
layer = [0]


def probe(qkv, B, S, H, scale, out, q_prescaled=True, **kw):
    q = qkv[:S, :H * 64].float().view(S, H, 64).transpose(0, 1)
    k = qkv[:S, H * 64:2 * H * 64].float().view(S, H, 64).transpose(0, 1)
    s = q @ k.transpose(1, 2)                        # [H, S, S], log2 units
    m0 = s[:, :, :64].amax(-1)
    grow = s.amax(-1) - m0                           # >= 0
    rowsum = torch.exp2(s - m0[..., None]).sum(-1)   # the kernel's row sum relative to m0
    bad = (grow > 16) | (rowsum > 65504)
    nq = (S + 127) // 128
    badwg = torch.zeros(H, nq, dtype=torch.bool, device=s.device)
    for i in range(nq):
        badwg[:, i] = bad[:, 128 * i:128 * (i + 1)].any(-1)
    print(f"layer {layer[0]:2d}: max growth {grow.max().item():6.2f} log2 units, rows past 16: "
          f"{(grow > 16).float().mean().item():.4f}, workgroups repeating: {badwg.float().mean().item():.3f}",
          flush=True)
    layer[0] += 1
    return real(qkv, B, S, H, scale, out, q_prescaled=q_prescaled, **kw)


ops.attention = probe
m.forward_logits(pix)
torch.cuda.synchronize()
