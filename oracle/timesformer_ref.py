"""ORACLE — test infrastructure only, never the product path.

A plain-PyTorch fp32 CPU restatement of the reference's TimeSformer forward (divided
space-time attention), the third-party arithmetic the reference calls through
`TimesformerForVideoClassification` (`timesformer/timesformer_classifier/models/
timesformer_model.py:37-41` -> transformers):

  per-frame Conv2d 16x16 patch embed, CLS + pos      TF5/models/timesformer/modeling_timesformer.py:45-113
  + time embeddings, re-ordered patch-major/time-minor                                   :115-143
  12 x layer, divided branch                                                              :332-398
    temporal: LN -> qkv -> attention over T per patch -> output.dense -> temporal_dense -> +res
    spatial:  CLS repeated per frame, LN -> attention over 1 + patches per frame -> output.dense,
              CLS outputs averaged over frames, + residual
    MLP: LN -> fc1 -> exact GELU -> fc2 -> +res
  final LN, classifier(seq[:, 0])                      :471-578, 604-712

Pinned against tests/golden/timesformer_tiny.npz (hidden states) and
tests/golden/timesformer_full.json (TimeSformer-B 8f logits), both produced by the
installed HF transformers model in the build container (tools/make_goldens.py).

Allowed importers: tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import torch

from oracle.vivit_ref import layer_norm


def _attn(x, wqkv, bqkv, H):
    """TimesformerSelfAttention (:148-180): x [N, L, D] -> context [N, L, D]."""
    N, L, D = x.shape
    qkv = (x @ wqkv.T + bqkv).reshape(N, L, 3, H, D // H).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    a = torch.softmax((q @ k.transpose(-2, -1)) * (D // H) ** -0.5, dim=-1)
    return (a @ v).transpose(1, 2).reshape(N, L, D)


def timesformer_forward(sd: dict, cfg: dict, pixel_values: torch.Tensor, return_hidden: bool = False):
    """sd: HF-named fp32 tensors; pixel_values [B,T,3,H,W] fp32 -> logits [B, num_labels]."""
    D = cfg["hidden_size"]
    H = cfg["num_attention_heads"]
    P = cfg["patch_size"]
    eps = cfg.get("layer_norm_eps", 1e-6)
    B, T, C, Hh, Ww = pixel_values.shape
    pw = Ww // P
    n = (Hh // P) * pw
    e = "timesformer.embeddings."
    x = torch.nn.functional.conv2d(pixel_values.reshape(B * T, C, Hh, Ww), sd[e + "patch_embeddings.projection.weight"],
                                   sd[e + "patch_embeddings.projection.bias"], stride=P)
    x = x.flatten(2).transpose(1, 2)                                   # [B*T, n, D], frame-major
    x = torch.cat([sd[e + "cls_token"].expand(B * T, -1, -1), x], 1) + sd[e + "position_embeddings"]
    cls = x[:B, 0:1]                                                   # every row's CLS is cls + pos[0]
    x = x[:, 1:].reshape(B, T, n, D).permute(0, 2, 1, 3).reshape(B * n, T, D) + sd[e + "time_embeddings"]
    h = torch.cat([cls, x.reshape(B, n * T, D)], 1)                   # [B, 1 + n*T, D] patch-major, time-minor
    hidden = [h]
    for i in range(cfg["num_hidden_layers"]):
        p = f"timesformer.encoder.layer.{i}."
        # temporal
        te = h[:, 1:].reshape(B * n, T, D)
        y = layer_norm(te, sd[p + "temporal_layernorm.weight"], sd[p + "temporal_layernorm.bias"], eps)
        y = _attn(y, sd[p + "temporal_attention.attention.qkv.weight"], sd[p + "temporal_attention.attention.qkv.bias"], H)
        y = y @ sd[p + "temporal_attention.output.dense.weight"].T + sd[p + "temporal_attention.output.dense.bias"]
        y = y.reshape(B, n * T, D) @ sd[p + "temporal_dense.weight"].T + sd[p + "temporal_dense.bias"]
        te = h[:, 1:] + y                                              # [B, n*T, D]
        # spatial
        init_cls = h[:, 0:1]
        sp = te.reshape(B, n, T, D).permute(0, 2, 1, 3).reshape(B * T, n, D)
        sp = torch.cat([init_cls.repeat(1, T, 1).reshape(B * T, 1, D), sp], 1)
        y = layer_norm(sp, sd[p + "layernorm_before.weight"], sd[p + "layernorm_before.bias"], eps)
        y = _attn(y, sd[p + "attention.attention.qkv.weight"], sd[p + "attention.attention.qkv.bias"], H)
        y = y @ sd[p + "attention.output.dense.weight"].T + sd[p + "attention.output.dense.bias"]
        cls_res = y[:, 0].reshape(B, T, D).mean(1, keepdim=True)
        res = y[:, 1:].reshape(B, T, n, D).permute(0, 2, 1, 3).reshape(B, n * T, D)
        h = torch.cat([init_cls, te], 1) + torch.cat([cls_res, res], 1)
        # MLP
        y = layer_norm(h, sd[p + "layernorm_after.weight"], sd[p + "layernorm_after.bias"], eps)
        y = torch.nn.functional.gelu(y @ sd[p + "intermediate.dense.weight"].T + sd[p + "intermediate.dense.bias"])
        h = h + y @ sd[p + "output.dense.weight"].T + sd[p + "output.dense.bias"]
        hidden.append(h)
    seq = layer_norm(h, sd["timesformer.layernorm.weight"], sd["timesformer.layernorm.bias"], eps)
    logits = seq[:, 0] @ sd["classifier.weight"].T + sd["classifier.bias"]
    if return_hidden:
        return logits, torch.stack(hidden)
    return logits
