"""Which weights set the fp16-operand ViViT-B logit error?  CPU emulation (tests/analysis/precision_probe.py's
forward): every rounding point fp16, then one weight group at a time kept fp32.
  python tests/analysis/w_probe.py [--clips 8]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import precision_probe as pp  # noqa: E402
from vclip_amd.weights import make_synthetic_clips, make_vivit_weights  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--clips", type=int, default=8)
a = ap.parse_args()
torch.set_num_threads(os.cpu_count())
cfg = dict(hidden_size=768, intermediate_size=3072, tubelet_size=[2, 16, 16], num_channels=3, num_frames=32,
           image_size=224, num_hidden_layers=12, num_labels=2, num_attention_heads=12, layer_norm_eps=1e-6)
sd = {k: torch.from_numpy(v) for k, v in make_vivit_weights(cfg, seed=0).items()}
pix = torch.from_numpy(make_synthetic_clips(a.clips, 32, 224, seed=1))
hf = torch.float16
half = {k: hf for k in pp.POINTS}
groups = {"embed": ["patch_embeddings"], "q|k|v": ["q_proj", "k_proj", "v_proj"], "o_proj": ["o_proj"],
          "fc1": ["mlp.fc1"], "fc2": ["mlp.fc2"], "layers 0-3": [f"layers.{i}." for i in range(4)],
          "layers 8-11": [f"layers.{i}." for i in range(8, 12)]}
ap2 = os.environ.get("WPROBE_GROUPS")
if ap2 == "embed_pix":
    groups = {"embed (+pix fp32)": ["patch_embeddings"], "embed+layer0 (+pix fp32)": ["patch_embeddings", "layers.0."]}
if ap2 == "l0":
    groups = {"embed+layer0 q|k|v (+pix fp32)": ["patch_embeddings", "layers.0.attention.q_proj",
                                                 "layers.0.attention.k_proj", "layers.0.attention.v_proj"],
              "embed+layer0 q|k|v+o (+pix fp32)": ["patch_embeddings", "layers.0.attention"],
              "layer0 (+pix fp32)": ["layers.0."],
              "embed+layers0-1 q|k|v (+pix fp32)": ["patch_embeddings", "layers.0.attention.q_proj",
                                                   "layers.0.attention.k_proj", "layers.0.attention.v_proj",
                                                   "layers.1.attention.q_proj", "layers.1.attention.k_proj",
                                                   "layers.1.attention.v_proj"]}
with torch.no_grad():
    ref = pp.forward(sd, cfg, pix, {k: None for k in pp.POINTS})
    for name, pats in groups.items():
        # pre-round every weight except the group to fp16 and run with w = fp32 (no further rounding)
        sd2 = {k: (v.to(hf).float() if v.dim() >= 2 and "position" not in k and "cls_token" not in k and
                   "classifier" not in k and not any(p in k for p in pats) else v) for k, v in sd.items()}
        got = pp.forward(sd2, cfg, pix, dict(half, w=None, **({"pix": None} if "pix" in name else {})))
        print(f"all fp16, {name:12s} weights fp32: max|err| {float((got - ref).abs().max()):.3e}", flush=True)
