"""Locate non-finite / wrong rows of the attention kernel on the score-scale test case."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops
from oracle.vivit_ref import attention_ref


def bf(x):
    return x.to(torch.bfloat16)


for mag in [4.0, 12.0]:
    B, S, H = 2, 777, 2
    g = torch.Generator().manual_seed(int(mag * 100))
    rows = (B - 1) * S + (S + 63) // 64 * 64 + 64
    qkv = torch.randn(rows, 3 * H * 64, generator=g)
    qkv[:, : 2 * H * 64] *= mag
    ramp = torch.linspace(0.2, 1.8, S).repeat(B)
    qkv[: B * S, H * 64: 2 * H * 64] *= ramp[:, None]
    qkv = bf(qkv)
    c = 0.125 * 1.4426950408889634
    qkv[:, : H * 64] = bf(qkv[:, : H * 64].float() * c)
    out = torch.zeros(rows, H * 64, dtype=torch.bfloat16, device="cuda")
    ops.attention(qkv.cuda(), B, S, H, 0.125, out, q_prescaled=True)
    q = qkv[: B * S].float().view(B, S, 3, H, 64)
    ref = attention_ref(q[:, :, 0].transpose(1, 2) / c, q[:, :, 1].transpose(1, 2), q[:, :, 2].transpose(1, 2), 0.125)
    ref = ref.transpose(1, 2).reshape(B, S, H, 64)
    o = out[: B * S].float().cpu().view(B, S, H, 64)
    bad = ~torch.isfinite(o)
    err = (o - ref).abs().nan_to_num(1e9)
    print(f"mag {mag}: nonfinite {int(bad.sum())}, rows with err>0.03: {int((err.amax(-1) > 0.03).sum())}")
    idx = (err.amax(-1) > 0.03).nonzero()
    for b_, s_, h_ in idx[:12].tolist():
        print("  b", b_, "q", s_, "h", h_, "qblk", s_ // 128, "wave", (s_ % 128) // 32, "lane", s_ % 32,
              "err", float(err[b_, s_, h_].max()), "vals", o[b_, s_, h_, :4].tolist(), "ref", ref[b_, s_, h_, :4].tolist())
    if idx.numel():
        print("  q rows hist:", torch.bincount(idx[:, 1] // 32).nonzero().flatten().tolist()[:40])
