"""ORACLE — test infrastructure only, never the product path.

A plain-PyTorch fp32 CPU restatement of the reference's ViViT forward (the third-party
arithmetic the reference calls through `VivitForVideoClassification`,
`vivit_transformer/vivit_classifier/models/vivit_model.py:37` -> transformers):

  tubelet Conv3d k=s=(2,16,16)      TF5/models/vivit/modeling_vivit.py:39-67
  CLS concat + position embeddings  TF5/.../modeling_vivit.py:126-146
  12 x pre-LN layer (eps 1e-6)      TF5/.../modeling_vivit.py:242-271
    joint attention, scale d^-1/2, fp32 softmax   :149-223
    MLP fc1 -> gelu_fast -> fc2     :226-239, TF5/activations.py (FastGELUActivation)
  final LN, classifier(seq[:, 0])   TF5/.../modeling_vivit.py:418-431, 462-566

Pinned against tests/golden/vivit_tiny.npz (full hidden states) and
tests/golden/vivit_full.json (ViViT-B/16x2 32f logits), both produced by the installed
HF transformers model in the build container (tools/make_goldens.py).

Allowed importers: tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import math

import torch


def gelu_fast(x: torch.Tensor) -> torch.Tensor:
    # 0.5 x (1 + tanh(0.7978845608 x (1 + 0.044715 x^2)))   (TF5/activations.py FastGELUActivation)
    return 0.5 * x * (1.0 + torch.tanh(x * 0.7978845608 * (1.0 + 0.044715 * x * x)))


def layer_norm(x, w, b, eps):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


def vivit_forward(sd: dict, cfg: dict, pixel_values: torch.Tensor, return_hidden: bool = False):
    """sd: HF-named fp32 tensors; pixel_values [B,T,3,H,W] fp32 -> logits [B, num_labels]."""
    D = cfg["hidden_size"]
    H = cfg["num_attention_heads"]
    hd = D // H
    eps = cfg.get("layer_norm_eps", 1e-6)
    kt, kh, kw = cfg["tubelet_size"]
    B, T, C, Hh, Ww = pixel_values.shape
    x = pixel_values.transpose(1, 2)  # [B,C,T,H,W]
    w = sd["vivit.embeddings.patch_embeddings.projection.weight"]
    emb = torch.nn.functional.conv3d(x, w, sd["vivit.embeddings.patch_embeddings.projection.bias"],
                                     stride=(kt, kh, kw))
    emb = emb.flatten(2).transpose(1, 2)  # [B, n, D], token order t, h, w
    cls = sd["vivit.embeddings.cls_token"].expand(B, -1, -1)
    h = torch.cat([cls, emb], dim=1) + sd["vivit.embeddings.position_embeddings"]
    hidden = [h]
    S = h.shape[1]
    scale = hd ** -0.5
    for i in range(cfg["num_hidden_layers"]):
        p = f"vivit.layers.{i}."
        r = h
        y = layer_norm(h, sd[p + "layernorm_before.weight"], sd[p + "layernorm_before.bias"], eps)

        def proj(nm, t):
            return t @ sd[p + f"attention.{nm}.weight"].T + sd[p + f"attention.{nm}.bias"]

        q = proj("q_proj", y).view(B, S, H, hd).transpose(1, 2)
        k = proj("k_proj", y).view(B, S, H, hd).transpose(1, 2)
        v = proj("v_proj", y).view(B, S, H, hd).transpose(1, 2)
        a = torch.softmax((q @ k.transpose(2, 3)) * scale, dim=-1, dtype=torch.float32)
        o = (a @ v).transpose(1, 2).reshape(B, S, D)
        h = proj("o_proj", o) + r
        r = h
        y = layer_norm(h, sd[p + "layernorm_after.weight"], sd[p + "layernorm_after.bias"], eps)
        y = gelu_fast(y @ sd[p + "mlp.fc1.weight"].T + sd[p + "mlp.fc1.bias"])
        h = y @ sd[p + "mlp.fc2.weight"].T + sd[p + "mlp.fc2.bias"] + r
        hidden.append(h)
    seq = layer_norm(h, sd["vivit.layernorm.weight"], sd["vivit.layernorm.bias"], eps)
    logits = seq[:, 0, :] @ sd["classifier.weight"].T + sd["classifier.bias"]
    if return_hidden:
        return logits, torch.stack(hidden)
    return logits


def attention_ref(q, k, v, scale=None):
    """Joint attention on [B,H,S,d] fp32 (TF5/.../modeling_vivit.py:149-174)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    a = torch.softmax((q.float() @ k.float().transpose(-1, -2)) * scale, dim=-1, dtype=torch.float32)
    return a @ v.float()
