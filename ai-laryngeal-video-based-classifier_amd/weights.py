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


def swin3d_param_shapes(cfg: dict) -> "OrderedDict[str, tuple]":
    """Parameter names and shapes of torchvision `swin3d_t` with the reference's replaced head
    (videoswintransformer/swin_video_classifier/models/swin3d.py:24-44), in a fixed order.
    The relative_position_index buffers are not parameters (rebuilt from the window size)."""
    C0 = cfg["embed_dim"]
    pt, ph, pw = cfg["patch_size"]
    wt, wh, ww = cfg["window_size"]
    nbias = (2 * wt - 1) * (2 * wh - 1) * (2 * ww - 1)
    s = OrderedDict()
    s["patch_embed.proj.weight"] = (C0, 3, pt, ph, pw)
    s["patch_embed.proj.bias"] = (C0,)
    s["patch_embed.norm.weight"] = (C0,)
    s["patch_embed.norm.bias"] = (C0,)
    for st, depth in enumerate(cfg["depths"]):
        C = C0 * 2 ** st
        heads = cfg["num_heads"][st]
        hid = int(C * cfg.get("mlp_ratio", 4.0))
        for i in range(depth):
            p = f"features.{2 * st}.{i}."
            s[p + "norm1.weight"] = (C,)
            s[p + "norm1.bias"] = (C,)
            s[p + "attn.relative_position_bias_table"] = (nbias, heads)
            s[p + "attn.qkv.weight"] = (3 * C, C)
            s[p + "attn.qkv.bias"] = (3 * C,)
            s[p + "attn.proj.weight"] = (C, C)
            s[p + "attn.proj.bias"] = (C,)
            s[p + "norm2.weight"] = (C,)
            s[p + "norm2.bias"] = (C,)
            s[p + "mlp.0.weight"] = (hid, C)
            s[p + "mlp.0.bias"] = (hid,)
            s[p + "mlp.3.weight"] = (C, hid)
            s[p + "mlp.3.bias"] = (C,)
        if st < len(cfg["depths"]) - 1:
            p = f"features.{2 * st + 1}."
            s[p + "reduction.weight"] = (2 * C, 4 * C)
            s[p + "norm.weight"] = (4 * C,)
            s[p + "norm.bias"] = (4 * C,)
    Cf = C0 * 2 ** (len(cfg["depths"]) - 1)
    s["norm.weight"] = (Cf,)
    s["norm.bias"] = (Cf,)
    s["head.weight"] = (cfg.get("num_classes", 2), Cf)
    s["head.bias"] = (cfg.get("num_classes", 2),)
    return s


def make_swin3d_weights(cfg: dict, seed: int = 0, std: float = 0.02) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.RandomState(seed)
    out = OrderedDict()
    for name, shape in swin3d_param_shapes(cfg).items():
        w = rng.standard_normal(shape) * std
        if name.endswith("norm.weight") or name.endswith("norm1.weight") or name.endswith("norm2.weight"):
            w = w + 1.0
        out[name] = np.ascontiguousarray(w.astype(np.float32))
    return out


def resnet3d_param_shapes(cfg: dict) -> "OrderedDict[str, tuple]":
    """Parameter / BatchNorm-buffer names and shapes of pytorchvideo `create_resnet` as the
    reference configures it (resnet50-3d-video/video_classifier/models/resnet3d.py:8-45)."""
    s = OrderedDict()

    def bn(pre, c):
        for k in ("weight", "bias", "running_mean", "running_var"):
            s[f"{pre}.{k}"] = (c,)

    d0 = cfg["stem_dim"]
    s["blocks.0.conv.weight"] = (d0, 3) + tuple(cfg.get("stem_kernel", (3, 7, 7)))
    bn("blocks.0.norm", d0)
    din, dout = d0, d0 * 4
    for st, depth in enumerate(cfg["depths"]):
        inner = dout // 4
        ka = cfg["conv_a_kernels"][st]
        for i in range(depth):
            p = f"blocks.{st + 1}.res_blocks.{i}."
            cin = din if i == 0 else dout
            if i == 0 and (cin != dout or cfg["spatial_strides"][st] != 1):
                s[p + "branch1_conv.weight"] = (dout, cin, 1, 1, 1)
                bn(p + "branch1_norm", dout)
            s[p + "branch2.conv_a.weight"] = (inner, cin) + tuple(ka)
            bn(p + "branch2.norm_a", inner)
            s[p + "branch2.conv_b.weight"] = (inner, inner, 1, 3, 3)
            bn(p + "branch2.norm_b", inner)
            s[p + "branch2.conv_c.weight"] = (dout, inner, 1, 1, 1)
            bn(p + "branch2.norm_c", dout)
        din, dout = dout, dout * 2
    if cfg.get("num_classes", 2):
        s["blocks.5.proj.weight"] = (cfg.get("num_classes", 2), din)
        s["blocks.5.proj.bias"] = (cfg.get("num_classes", 2),)
    return s


def make_resnet3d_weights(cfg: dict, seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """Convs ~ N(0, 2/fan_in) (He), BN gamma = 1 + N(0, .02), beta / running_mean ~ N(0, .02),
    running_var = 1 + |N(0, .02)|; the last BN of every residual branch gets gamma scaled by
    0.2 so the 16-block residual stream stays O(1) with random weights."""
    rng = np.random.RandomState(seed)
    out = OrderedDict()
    for name, shape in resnet3d_param_shapes(cfg).items():
        if name.endswith("conv.weight") or name.endswith("conv_a.weight") or name.endswith("conv_b.weight") or \
                name.endswith("conv_c.weight"):
            fan_in = int(np.prod(shape[1:]))
            w = rng.standard_normal(shape) * np.sqrt(2.0 / fan_in)
        elif name.endswith("running_var"):
            w = 1.0 + np.abs(rng.standard_normal(shape) * 0.02)
        elif name.endswith("norm.weight") or name.endswith("norm_a.weight") or name.endswith("norm_b.weight") or \
                name.endswith("norm_c.weight"):
            w = 1.0 + rng.standard_normal(shape) * 0.02
            if name.endswith("norm_c.weight"):
                w = w * 0.2
        else:
            w = rng.standard_normal(shape) * 0.02
        out[name] = np.ascontiguousarray(w.astype(np.float32))
    return out


# torchvision resnet50 (the per-frame feature extractor of resnet50-2d-lstm/src/models/model.py:9-12,
# nn.Sequential(children()[:-1]) -> keys "resnet50.<child>...") <-> the pytorchvideo-style names
# the shared conv path packs (kt = 1 kernels)
RESNET50_2D = dict(depths=(3, 4, 6, 3), stem_dim=64, conv_a_kernels=((1, 1, 1),) * 4, spatial_strides=(1, 2, 2, 2),
                   num_classes=0, bn_eps=1e-5, stem_kernel=(1, 7, 7), stem_pad=(0, 3, 3))


def torchvision_resnet50_to_blocks(name: str):
    """'resnet50.4.0.conv1.weight' -> 'blocks.1.res_blocks.0.branch2.conv_a.weight' (None if not a
    ResNet key).  Children: 0 conv1, 1 bn1, 4..7 layer1..4 (Bottleneck v1.5: stride on conv2)."""
    parts = name.split(".")
    if parts[0] != "resnet50":
        return None
    child = int(parts[1])
    if child == 0:
        return "blocks.0.conv." + parts[-1]
    if child == 1:
        return "blocks.0.norm." + parts[-1]
    stage, blk, mod = child - 3, parts[2], parts[3]
    pre = f"blocks.{stage}.res_blocks.{blk}."
    if mod == "downsample":
        return pre + ("branch1_conv." if parts[4] == "0" else "branch1_norm.") + parts[-1]
    m = {"conv1": "branch2.conv_a", "bn1": "branch2.norm_a", "conv2": "branch2.conv_b", "bn2": "branch2.norm_b",
         "conv3": "branch2.conv_c", "bn3": "branch2.norm_c"}[mod]
    return pre + m + "." + parts[-1]


def resnet50_lstm_param_shapes(hidden: int = 256, layers: int = 2) -> "OrderedDict[str, tuple]":
    """Reference VideoResNet50LSTM state_dict names / shapes (resnet50-2d-lstm/src/models/model.py)."""
    inv = {}
    s = OrderedDict()
    for n, shp in resnet3d_param_shapes(RESNET50_2D).items():
        inv[n] = shp
    # torchvision order: conv1, bn1, layer1..4
    for n, shp in inv.items():
        tv = blocks_to_torchvision_resnet50(n)
        s[tv] = shp[:2] + shp[3:] if len(shp) == 5 else shp  # 2D conv weights drop the kt = 1 axis
    for l in range(layers):
        din = 2048 if l == 0 else hidden
        s[f"lstm.weight_ih_l{l}"] = (4 * hidden, din)
        s[f"lstm.weight_hh_l{l}"] = (4 * hidden, hidden)
        s[f"lstm.bias_ih_l{l}"] = (4 * hidden,)
        s[f"lstm.bias_hh_l{l}"] = (4 * hidden,)
    s["classifier.0.weight"] = (64, hidden)
    s["classifier.0.bias"] = (64,)
    s["classifier.3.weight"] = (1, 64)
    s["classifier.3.bias"] = (1,)
    return s


def blocks_to_torchvision_resnet50(name: str) -> str:
    parts = name.split(".")
    if parts[1] == "0":
        return ("resnet50.0." if parts[2] == "conv" else "resnet50.1.") + parts[-1]
    stage, blk = int(parts[1]), parts[3]
    pre = f"resnet50.{stage + 3}.{blk}."
    if parts[4].startswith("branch1"):
        return pre + ("downsample.0." if parts[4] == "branch1_conv" else "downsample.1.") + parts[-1]
    m = {"conv_a": "conv1", "norm_a": "bn1", "conv_b": "conv2", "norm_b": "bn2", "conv_c": "conv3", "norm_c": "bn3"}[parts[5]]
    return pre + m + "." + parts[-1]


def make_resnet50_lstm_weights(seed: int = 0, hidden: int = 256) -> "OrderedDict[str, np.ndarray]":
    """ResNet part as make_resnet3d_weights (He convs, near-identity BN); LSTM / classifier ~
    U(-1/sqrt(hidden), 1/sqrt(hidden)) like torch's default init."""
    base = make_resnet3d_weights(RESNET50_2D, seed=seed)
    rng = np.random.RandomState(seed + 1)
    out = OrderedDict()
    for n, shp in resnet50_lstm_param_shapes(hidden).items():
        if n.startswith("resnet50."):
            b = base[torchvision_resnet50_to_blocks(n)]
            out[n] = np.ascontiguousarray(b.reshape(shp))
        else:
            k = 1.0 / np.sqrt(hidden if n.startswith("lstm") else shp[-1])
            out[n] = np.ascontiguousarray(rng.uniform(-k, k, shp).astype(np.float32))
    return out


def make_synthetic_video(batch: int, num_frames: int, image_size: int, seed: int = 1) -> np.ndarray:
    """[B, 3, T, H, W] f32 (the torchvision video-model input layout, swin trainer.py:116):
    the uint8 frames of make_synthetic_frames through the Swin/ResNet3D transform's
    Normalize(0.45, 0.225) on x/255 (resize/crop skipped: frames are 224^2)."""
    f = make_synthetic_frames(batch, num_frames, image_size, seed).astype(np.float32)
    x = (f / np.float32(255.0) - np.float32(0.45)) / np.float32(0.225)
    return np.ascontiguousarray(x.transpose(0, 4, 1, 2, 3))


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
