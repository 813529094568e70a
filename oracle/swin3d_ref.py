"""ORACLE — test infrastructure only, never the product path.

A plain-PyTorch fp32 CPU restatement of Video Swin-T as the reference builds it:
`videoswintransformer/swin_video_classifier/models/swin3d.py:7-53` calls torchvision's
`swin3d_t(weights=...)` and replaces `model.head` with `nn.Linear(768, num_classes)`
(:43-44); the model is called as `model(f32[B,3,T,H,W])` (trainer.py:116).

PARITY UNPINNED: torchvision is not installed in this image and its source is nowhere on
disk, so this restatement follows torchvision's published algorithm for
`torchvision.models.video.swin_transformer` (torchvision 0.15-0.21; the reference's
requirements.txt does not pin torchvision) — it cannot be checked against the library
itself here.  What it restates:

  PatchEmbed3d: Conv3d k=s=(2,4,4) 3->96, channels-last, LayerNorm(eps 1e-5)
  4 stages, depths (2,2,6,2), heads (3,6,12,24), head_dim 32, window (8,7,7),
    block i of a stage shifted by (4,3,3) when i is odd; a window / shift dimension is
    clamped to the feature size (and the shift to 0) where size <= window
    (_get_window_and_shift_size); the relative-position index of the FULL window is
    sliced [:vol, :vol] when the window shrinks (torchvision's behaviour, kept);
  block: x + attn(LN(x)), x + MLP(LN(x)) (Linear, exact GELU, Linear), LN eps 1e-5;
  ShiftedWindowAttention3d: zero-pad to whole windows, roll by -shift, partition,
    qkv Linear, q * d^-1/2, + relative_position_bias_table[index], shifted blocks add
    -100 between tokens of different shift regions (the t/h/w slice labelling of
    shifted_window_attention_3d), softmax, proj Linear, reverse partition, roll back, crop;
  PatchMerging between stages: concat of the (0::2,0::2), (1::2,0::2), (0::2,1::2),
    (1::2,1::2) spatial neighbours (zero-padded to even H, W), LayerNorm(4C), Linear(4C,2C, no bias);
  final LayerNorm(768), mean over (T, H, W), head Linear(768, num_classes).

Parameter names follow torchvision's state_dict (patch_embed.*, features.{2s}.{i}.*,
features.{2s+1}.* (PatchMerging), norm.*, head.*).

Allowed importers: tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

SWIN3D_T = dict(patch_size=(2, 4, 4), embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24),
                window_size=(8, 7, 7), mlp_ratio=4.0, num_classes=2, layer_norm_eps=1e-5)


def relative_position_index(window_size):
    """torchvision ShiftedWindowAttention3d.define_relative_position_index."""
    wt, wh, ww = window_size
    coords = torch.stack(torch.meshgrid(torch.arange(wt), torch.arange(wh), torch.arange(ww), indexing="ij"))
    cf = torch.flatten(coords, 1)
    rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += wt - 1
    rel[:, :, 1] += wh - 1
    rel[:, :, 2] += ww - 1
    rel[:, :, 0] *= (2 * wh - 1) * (2 * ww - 1)
    rel[:, :, 1] *= 2 * ww - 1
    return rel.sum(-1)


def window_and_shift(size_thw, window_size, shift_size):
    """torchvision _get_window_and_shift_size."""
    w, s = list(window_size), list(shift_size)
    for i in range(3):
        if size_thw[i] <= w[i]:
            w[i] = size_thw[i]
            s[i] = 0
    return w, s


def relative_position_bias(table, full_window, window):
    """[heads, vol, vol] bias: table[index_full[:vol,:vol]] (torchvision _get_relative_position_bias)."""
    vol = window[0] * window[1] * window[2]
    idx = relative_position_index(full_window)[:vol, :vol].flatten()
    return table[idx].view(vol, vol, -1).permute(2, 0, 1).contiguous()


def shift_region_labels(padded_thw, window, shift):
    """Per-position shift-region label of shifted_window_attention_3d's attn_mask (t/h/w slices,
    later slices overwrite earlier ones), [Tp, Hp, Wp]."""
    tp, hp, wp = padded_thw
    lab = torch.zeros((tp, hp, wp))
    count = 0
    sl = [((0, -window[d]), (-window[d], -shift[d]), (-shift[d], None)) for d in range(3)]
    for t in sl[0]:
        for h in sl[1]:
            for w in sl[2]:
                lab[t[0]:t[1], h[0]:h[1], w[0]:w[1]] = count
                count += 1
    return lab


def window_attention_3d(x, p, prefix, num_heads, full_window, shift_size):
    """ShiftedWindowAttention3d.forward on x [B, T, H, W, C] (already LayerNorm-ed)."""
    b, t, h, w, c = x.shape
    window, shift = window_and_shift((t, h, w), full_window, shift_size)
    bias = relative_position_bias(p[prefix + "relative_position_bias_table"], full_window, window)
    pad = [(window[i] - (s % window[i])) % window[i] for i, s in enumerate((t, h, w))]
    x = F.pad(x, (0, 0, 0, pad[2], 0, pad[1], 0, pad[0]))
    _, tp, hp, wp, _ = x.shape
    if sum(shift) > 0:
        x = torch.roll(x, shifts=(-shift[0], -shift[1], -shift[2]), dims=(1, 2, 3))
    nw = (tp // window[0]) * (hp // window[1]) * (wp // window[2])
    vol = window[0] * window[1] * window[2]
    x = x.view(b, tp // window[0], window[0], hp // window[1], window[1], wp // window[2], window[2], c)
    x = x.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(b * nw, vol, c)
    qkv = F.linear(x, p[prefix + "qkv.weight"], p[prefix + "qkv.bias"])
    qkv = qkv.reshape(x.size(0), vol, 3, num_heads, c // num_heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * (c // num_heads) ** -0.5
    attn = q.matmul(k.transpose(-2, -1)) + bias.unsqueeze(0)
    if sum(shift) > 0:
        m = shift_region_labels((tp, hp, wp), window, shift)
        m = m.view(tp // window[0], window[0], hp // window[1], window[1], wp // window[2], window[2])
        m = m.permute(0, 2, 4, 1, 3, 5).reshape(nw, vol)
        m = m.unsqueeze(1) - m.unsqueeze(2)
        m = m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)
        attn = attn.view(b, nw, num_heads, vol, vol) + m.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, num_heads, vol, vol)
    attn = F.softmax(attn, dim=-1)
    x = attn.matmul(v).transpose(1, 2).reshape(b * nw, vol, c)
    x = F.linear(x, p[prefix + "proj.weight"], p[prefix + "proj.bias"])
    x = x.view(b, tp // window[0], hp // window[1], wp // window[2], window[0], window[1], window[2], c)
    x = x.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(b, tp, hp, wp, c)
    if sum(shift) > 0:
        x = torch.roll(x, shifts=(shift[0], shift[1], shift[2]), dims=(1, 2, 3))
    return x[:, :t, :h, :w, :].contiguous()


def patch_merging(x, p, prefix, eps):
    """torchvision PatchMerging on [..., H, W, C]."""
    H, W = x.shape[-3], x.shape[-2]
    x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2))
    x = torch.cat([x[..., 0::2, 0::2, :], x[..., 1::2, 0::2, :], x[..., 0::2, 1::2, :], x[..., 1::2, 1::2, :]], -1)
    x = F.layer_norm(x, (x.shape[-1],), p[prefix + "norm.weight"], p[prefix + "norm.bias"], eps)
    return F.linear(x, p[prefix + "reduction.weight"])


def swin3d_forward(p: dict, cfg: dict, video: torch.Tensor, return_stages: bool = False):
    """p: torchvision-named fp32 tensors; video [B, 3, T, H, W] fp32 -> logits [B, num_classes]."""
    eps = cfg.get("layer_norm_eps", 1e-5)
    pt, ph, pw = cfg["patch_size"]
    b, _, t, h, w = video.shape
    pad = [(k - (s % k)) % k for k, s in zip((pt, ph, pw), (t, h, w))]
    x = F.pad(video, (0, pad[2], 0, pad[1], 0, pad[0]))
    x = F.conv3d(x, p["patch_embed.proj.weight"], p["patch_embed.proj.bias"], stride=(pt, ph, pw))
    x = x.permute(0, 2, 3, 4, 1)
    x = F.layer_norm(x, (x.shape[-1],), p["patch_embed.norm.weight"], p["patch_embed.norm.bias"], eps)
    stages = [x]
    win = tuple(cfg["window_size"])
    for s, depth in enumerate(cfg["depths"]):
        heads = cfg["num_heads"][s]
        for i in range(depth):
            pre = f"features.{2 * s}.{i}."
            shift = [0 if i % 2 == 0 else k // 2 for k in win]
            y = F.layer_norm(x, (x.shape[-1],), p[pre + "norm1.weight"], p[pre + "norm1.bias"], eps)
            x = x + window_attention_3d(y, p, pre + "attn.", heads, win, shift)
            y = F.layer_norm(x, (x.shape[-1],), p[pre + "norm2.weight"], p[pre + "norm2.bias"], eps)
            y = F.gelu(F.linear(y, p[pre + "mlp.0.weight"], p[pre + "mlp.0.bias"]))
            x = x + F.linear(y, p[pre + "mlp.3.weight"], p[pre + "mlp.3.bias"])
        if s < len(cfg["depths"]) - 1:
            x = patch_merging(x, p, f"features.{2 * s + 1}.", eps)
        stages.append(x)
    x = F.layer_norm(x, (x.shape[-1],), p["norm.weight"], p["norm.bias"], eps)
    x = x.mean(dim=(1, 2, 3))
    logits = F.linear(x, p["head.weight"], p["head.bias"])
    if return_stages:
        return logits, stages
    return logits
