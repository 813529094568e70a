"""Deterministic synthetic weights / inputs shared by goldens, tests and bench.

There is no network, so pretrained checkpoints (`google/vivit-b-16x2-kinetics400`,
reference `vivit_transformer/vivit_classifier/models/vivit_model.py:37`) cannot be
fetched.  Every consumer instead regenerates the same fp32 weights from a seed with
numpy's legacy `RandomState` stream (stable across numpy versions), in the HF
transformers-5 key naming of `VivitForVideoClassification`
(TF5/models/vivit/modeling_vivit.py:39-271, 462-566).  SURVEY.md §8(d) fixes the
distributions: Linear/Conv ~ N(0, 0.02), LayerNorm gamma = 1 + N(0, 0.02),
beta/bias/cls/pos ~ N(0, 0.02).  Seeds: 0 for weights, 1 for inputs.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np


def vivit_param_shapes(cfg: dict) -> "OrderedDict[str, tuple]":
    """Parameter names and shapes of HF VivitForVideoClassification (2 labels), in a fixed order."""
    D = cfg["hidden_size"]
    I = cfg["intermediate_size"]
    kt, kh, kw = cfg["tubelet_size"]
    C = cfg.get("num_channels", 3)
    n_tok = (cfg["num_frames"] // kt) * (cfg["image_size"] // kh) * (cfg["image_size"] // kw)
    L = cfg["num_hidden_layers"]
    nl = cfg.get("num_labels", 2)
    s = OrderedDict()
    s["vivit.embeddings.cls_token"] = (1, 1, D)
    s["vivit.embeddings.position_embeddings"] = (1, n_tok + 1, D)
    s["vivit.embeddings.patch_embeddings.projection.weight"] = (D, C, kt, kh, kw)
    s["vivit.embeddings.patch_embeddings.projection.bias"] = (D,)
    for i in range(L):
        p = f"vivit.layers.{i}."
        for nm in ("q_proj", "k_proj", "v_proj", "o_proj"):
            s[p + f"attention.{nm}.weight"] = (D, D)
            s[p + f"attention.{nm}.bias"] = (D,)
        s[p + "layernorm_before.weight"] = (D,)
        s[p + "layernorm_before.bias"] = (D,)
        s[p + "layernorm_after.weight"] = (D,)
        s[p + "layernorm_after.bias"] = (D,)
        s[p + "mlp.fc1.weight"] = (I, D)
        s[p + "mlp.fc1.bias"] = (I,)
        s[p + "mlp.fc2.weight"] = (D, I)
        s[p + "mlp.fc2.bias"] = (D,)
    s["vivit.layernorm.weight"] = (D,)
    s["vivit.layernorm.bias"] = (D,)
    s["classifier.weight"] = (nl, D)
    s["classifier.bias"] = (nl,)
    return s


def make_vivit_weights(cfg: dict, seed: int = 0, std: float = 0.02) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.RandomState(seed)
    out = OrderedDict()
    for name, shape in vivit_param_shapes(cfg).items():
        w = rng.standard_normal(shape) * std
        if name.endswith("norm_before.weight") or name.endswith("norm_after.weight") or name == "vivit.layernorm.weight":
            w = w + 1.0
        out[name] = np.ascontiguousarray(w.astype(np.float32))
    return out


def timesformer_param_shapes(cfg: dict) -> "OrderedDict[str, tuple]":
    """Parameter names and shapes of HF TimesformerForVideoClassification (divided space-time,
    TF5/models/timesformer/modeling_timesformer.py:67-145, 148-398, 462-712), fixed order."""
    D = cfg["hidden_size"]
    I = cfg["intermediate_size"]
    P = cfg["patch_size"]
    C = cfg.get("num_channels", 3)
    n_patch = (cfg["image_size"] // P) ** 2
    L = cfg["num_hidden_layers"]
    nl = cfg.get("num_labels", 2)
    s = OrderedDict()
    s["timesformer.embeddings.cls_token"] = (1, 1, D)
    s["timesformer.embeddings.position_embeddings"] = (1, n_patch + 1, D)
    s["timesformer.embeddings.time_embeddings"] = (1, cfg["num_frames"], D)
    s["timesformer.embeddings.patch_embeddings.projection.weight"] = (D, C, P, P)
    s["timesformer.embeddings.patch_embeddings.projection.bias"] = (D,)
    for i in range(L):
        p = f"timesformer.encoder.layer.{i}."
        for att in ("attention", "temporal_attention"):
            s[p + f"{att}.attention.qkv.weight"] = (3 * D, D)
            s[p + f"{att}.attention.qkv.bias"] = (3 * D,)
            s[p + f"{att}.output.dense.weight"] = (D, D)
            s[p + f"{att}.output.dense.bias"] = (D,)
        s[p + "intermediate.dense.weight"] = (I, D)
        s[p + "intermediate.dense.bias"] = (I,)
        s[p + "output.dense.weight"] = (D, I)
        s[p + "output.dense.bias"] = (D,)
        for ln in ("layernorm_before", "layernorm_after", "temporal_layernorm"):
            s[p + f"{ln}.weight"] = (D,)
            s[p + f"{ln}.bias"] = (D,)
        s[p + "temporal_dense.weight"] = (D, D)
        s[p + "temporal_dense.bias"] = (D,)
    s["timesformer.layernorm.weight"] = (D,)
    s["timesformer.layernorm.bias"] = (D,)
    s["classifier.weight"] = (nl, D)
    s["classifier.bias"] = (nl,)
    return s


def make_timesformer_weights(cfg: dict, seed: int = 0, std: float = 0.02) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.RandomState(seed)
    out = OrderedDict()
    for name, shape in timesformer_param_shapes(cfg).items():
        w = rng.standard_normal(shape) * std
        if name.endswith("norm_before.weight") or name.endswith("norm_after.weight") or \
                name.endswith("temporal_layernorm.weight") or name == "timesformer.layernorm.weight":
            w = w + 1.0
        out[name] = np.ascontiguousarray(w.astype(np.float32))
    return out


def make_synthetic_frames(batch: int, num_frames: int, image_size: int, seed: int = 1) -> np.ndarray:
    """uint8 decoded frames [B, T, H, W, 3] (the layout the reference dataset returns,
    vivit_transformer/vivit_classifier/data_config/dataset.py:268-291)."""
    rng = np.random.RandomState(seed)
    return rng.randint(0, 256, size=(batch, num_frames, image_size, image_size, 3)).astype(np.uint8)


# ViViT processor net affine: x*(1/127.5) - 1, then (x - 0.5)/0.5  ==>  x/63.75 - 3
# (transformers VivitImageProcessor rescale offset=True + normalize 0.5/0.5)
VIVIT_SCALE = np.float32(1.0 / 63.75)
VIVIT_SHIFT = np.float32(-3.0)


def frames_to_pixel_values(frames_u8: np.ndarray) -> np.ndarray:
    """[B,T,H,W,3] uint8 -> [B,T,3,H,W] float32 with the ViViT processor affine (crop/resize skipped:
    frames are already 224x224 as the dataset returns them)."""
    x = frames_u8.astype(np.float32) * VIVIT_SCALE + VIVIT_SHIFT
    return np.ascontiguousarray(x.transpose(0, 1, 4, 2, 3))


def make_synthetic_clips(batch: int, num_frames: int, image_size: int, seed: int = 1) -> np.ndarray:
    return frames_to_pixel_values(make_synthetic_frames(batch, num_frames, image_size, seed))


def sha256_state(sd) -> str:
    h = hashlib.sha256()
    for k in sd:
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k]).tobytes())
    return h.hexdigest()
