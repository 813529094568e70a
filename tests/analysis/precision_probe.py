"""Where does the ViViT-B logit error come from?  CPU experiment (no GPU).

Re-runs the fp32 oracle's arithmetic (oracle/vivit_ref.py) with the HIP path's rounding
points switched on one at a time: each point rounds to bf16 (the shipped path), to fp16, or
stays fp32.  Rounding points of the HIP forward:
  pix   im2col operand (pixel values)        w     every GEMM weight
  ln    LayerNorm output (GEMM A operand)    qkv   q|k|v GEMM output
  p     softmax numerator P before P.V       o     attention output (o_proj A operand)
  hid   GELU output (fc2 A operand)
Reports max |logit - fp32 logit| per configuration on B clips of ViViT-B/16x2 32x224^2.

  python tests/analysis/precision_probe.py [--clips 2] [--layers 12]
"""
import argparse
import itertools
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.vivit_ref import gelu_fast, layer_norm  # noqa: E402
from vclip_amd.weights import make_synthetic_clips, make_vivit_weights  # noqa: E402

POINTS = ["pix", "w", "ln", "qkv", "p", "o", "hid"]


def rnd(x, dt):
    return x if dt is None else x.to(dt).float()


def forward(sd, cfg, pix, rp):
    D, H = cfg["hidden_size"], cfg["num_attention_heads"]
    hd = D // H
    eps = cfg["layer_norm_eps"]
    W = {k: (rnd(v, rp["w"]) if v.dim() >= 2 and "position" not in k and "cls_token" not in k and
             "classifier" not in k else v) for k, v in sd.items()}
    B, T, C, Hh, Ww = pix.shape
    x = rnd(pix, rp["pix"]).transpose(1, 2)
    emb = torch.nn.functional.conv3d(x, W["vivit.embeddings.patch_embeddings.projection.weight"],
                                     sd["vivit.embeddings.patch_embeddings.projection.bias"], stride=(2, 16, 16))
    emb = emb.flatten(2).transpose(1, 2)
    h = torch.cat([sd["vivit.embeddings.cls_token"].expand(B, -1, -1), emb], 1) + sd["vivit.embeddings.position_embeddings"]
    S = h.shape[1]
    c = hd ** -0.5
    for i in range(cfg["num_hidden_layers"]):
        p = f"vivit.layers.{i}."
        r = h
        y = rnd(layer_norm(h, sd[p + "layernorm_before.weight"], sd[p + "layernorm_before.bias"], eps), rp["ln"])

        def proj(nm, t):
            return t @ W[p + f"attention.{nm}.weight"].T + sd[p + f"attention.{nm}.bias"]

        q = rnd(proj("q_proj", y), rp["qkv"]).view(B, S, H, hd).transpose(1, 2)
        k = rnd(proj("k_proj", y), rp["qkv"]).view(B, S, H, hd).transpose(1, 2)
        v = rnd(proj("v_proj", y), rp["qkv"]).view(B, S, H, hd).transpose(1, 2)
        s = (q @ k.transpose(2, 3)) * c
        m = s.amax(-1, keepdim=True)
        e = torch.exp(s - m)
        l = e.sum(-1, keepdim=True)
        o = (rnd(e, rp["p"]) @ v) / l
        o = rnd(o.transpose(1, 2).reshape(B, S, D), rp["o"])
        h = proj("o_proj", o) + r
        r = h
        y = rnd(layer_norm(h, sd[p + "layernorm_after.weight"], sd[p + "layernorm_after.bias"], eps), rp["ln"])
        y = rnd(gelu_fast(y @ W[p + "mlp.fc1.weight"].T + sd[p + "mlp.fc1.bias"]), rp["hid"])
        h = y @ W[p + "mlp.fc2.weight"].T + sd[p + "mlp.fc2.bias"] + r
    seq = layer_norm(h[:, :1], sd["vivit.layernorm.weight"], sd["vivit.layernorm.bias"], eps)
    return seq[:, 0, :] @ sd["classifier.weight"].T + sd["classifier.bias"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=2)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--fp16-ablate", action="store_true", help="all fp16, one point at a time back to fp32")
    ap.add_argument("--mixed", action="store_true", help="fp16 GEMMs with bf16 attention and the converse")
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    cfg = dict(hidden_size=768, intermediate_size=3072, tubelet_size=[2, 16, 16], num_channels=3, num_frames=32,
               image_size=224, num_hidden_layers=a.layers, num_labels=2, num_attention_heads=12, layer_norm_eps=1e-6)
    sd = {k: torch.from_numpy(v) for k, v in make_vivit_weights(cfg, seed=0).items()}
    pix = torch.from_numpy(make_synthetic_clips(a.clips, 32, 224, seed=1))
    bf, hf = torch.bfloat16, torch.float16
    with torch.no_grad():
        ref = forward(sd, cfg, pix, {k: None for k in POINTS})
        print("fp32 logits", ref.numpy().round(4).tolist(), flush=True)
        shipped = {k: bf for k in POINTS}
        if a.mixed:
            gemm16 = dict(shipped, pix=hf, w=hf, ln=hf, o=hf, hid=hf)   # attention operands q|k|v, P in bf16
            attn16 = dict(shipped, qkv=hf, p=hf)                          # GEMM operands in bf16
            for name, rp in (("fp16 GEMMs, bf16 attention", gemm16), ("bf16 GEMMs, fp16 attention", attn16),
                             ("fp16 GEMMs except embed", dict(gemm16, pix=bf, qkv=hf, p=hf)),
                             ("fp16 weights+o+hid, bf16 ln", dict(shipped, w=hf, o=hf, hid=hf, qkv=hf, p=hf))):
                got = forward(sd, cfg, pix, rp)
                print(f"{name:40s} max|err| {float((got - ref).abs().max()):.3e}", flush=True)
            return
        if a.fp16_ablate:
            half = {k: hf for k in POINTS}
            runs = [("all fp16", half)] + [(f"all fp16 except {k} fp32", dict(half, **{k: None})) for k in POINTS]
            runs += [("all fp16 except w+ln fp32", dict(half, w=None, ln=None)),
                     ("all fp16 except p+o fp32", dict(half, p=None, o=None))]
            for name, rp in runs:
                got = forward(sd, cfg, pix, rp)
                print(f"{name:40s} max|err| {float((got - ref).abs().max()):.3e}", flush=True)
            return
        runs = [("all bf16 (shipped rounding points)", shipped)]
        for k in POINTS:
            runs.append((f"all bf16 except {k} fp32", dict(shipped, **{k: None})))
        for k in POINTS:
            runs.append((f"only {k} bf16", dict({j: None for j in POINTS}, **{k: bf})))
        runs.append(("all bf16, p fp16", dict(shipped, p=hf)))
        runs.append(("all bf16, p+qkv fp16", dict(shipped, p=hf, qkv=hf)))
        runs.append(("all fp16", {k: hf for k in POINTS}))
        for name, rp in runs:
            t0 = time.time()
            got = forward(sd, cfg, pix, rp)
            print(f"{name:40s} max|err| {float((got - ref).abs().max()):.3e}  ({time.time() - t0:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
