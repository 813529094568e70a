"""Clip preprocessing on the GPU: drop-ins for the
reference's per-model input pipelines, applied to decoded uint8 frames already on the device.

* `vivit_preprocess` — transformers `VivitImageProcessor(num_frames, image_size=224,
  patch_size=16)` as the ViViT trainer / evaluator / inference use it
  (vivit_transformer/vivit_classifier/trainers/trainer.py:22-26, 62-95): Pillow BILINEAR resize
  of the shortest edge to 256 (uint8 result, bit-exact: Pillow's fixed-point two-pass
  resampler), centre crop 224, x * (1/127.5) - 1 then (x - 0.5) / 0.5  (= x / 63.75 - 3).
* `video_eval_transform` — pytorchvideo UniformTemporalSubsample(T) -> ShortSideScale(256) ->
  CenterCrop(224) -> Normalize(0.45, 0.225) of the Swin / ResNet3D / LSTM eval datasets
  (videoswintransformer/.../dataset.py:162-170; note the reference normalises the 0..255
  values WITHOUT a /255 there, reproduced as is), or with div255=True the inference scripts'
  (x/255 - 0.45)/0.225 (resnet50-3d-video/inference.py:382-394); output [B, 3, T, 224, 224].
* `timesformer_preprocess` — the AutoImageProcessor of timesformer/.../trainer.py:21-24 with size
  and crop forced to 224: a no-op resize/crop, x/255, then (x - mean)/std (mean/std from the hub
  config: not retrievable offline, passed in; default ImageNet 0.45/0.225 per SURVEY §8 a6).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib
from .ops import _dev, _need, _p, _stream

PRECISION_BITS = 32 - 8 - 2


def pil_bilinear_coeffs(in_size: int, out_size: int):
    """Pillow Resample.c precompute_coeffs(BILINEAR, box=(0, in_size)) + normalize_coeffs_8bpc:
    returns (bounds int32 [out, 2], coeffs int32 [out, ksize], ksize)."""
    support_base = 1.0  # bilinear filter support
    scale = filterscale = float(in_size) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = support_base * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, ksize), dtype=np.float64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w = 1.0 - t if t < 1.0 else 0.0
            kk[xx, x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                kk[xx, x] /= ww
        bounds[xx] = (xmin, xmax)
    one = float(1 << PRECISION_BITS)
    coef = np.where(kk < 0, np.trunc(-0.5 + kk * one), np.trunc(0.5 + kk * one)).astype(np.int32)
    return bounds, coef, ksize


_coef_cache = {}


def _coef_dev(in_size, out_size, device):
    key = (in_size, out_size, str(device))
    if key not in _coef_cache:
        b, c, k = pil_bilinear_coeffs(in_size, out_size)
        _coef_cache[key] = (torch.from_numpy(b).to(device), torch.from_numpy(c).to(device), k)
    return _coef_cache[key]


def pil_resize_u8(frames: torch.Tensor, out_hw) -> torch.Tensor:
    """frames u8 [N, H, W, C] (device) -> u8 [N, H2, W2, C] = PIL Image.resize((W2, H2), BILINEAR),
    bit-exact (Pillow resizes horizontally first, then vertically; a pass is skipped when that
    dimension does not change)."""
    _dev(frames)
    _need(frames.dtype == torch.uint8 and frames.dim() == 4 and frames.is_contiguous(), "pil_resize_u8: u8 [N,H,W,C]")
    N, H, W, C = frames.shape
    H2, W2 = out_hw
    x = frames
    if W2 != W:
        b, c, k = _coef_dev(W, W2, frames.device)
        y = torch.empty((N, H, W2, C), dtype=torch.uint8, device=frames.device)
        _lib.call("vc_resample_u8", _p(x), N, H, W, C, 0, W2, _p(b), _p(c), k, _p(y), _stream(x))
        x, W = y, W2
    if H2 != H:
        b, c, k = _coef_dev(H, H2, frames.device)
        y = torch.empty((N, H2, W, C), dtype=torch.uint8, device=frames.device)
        _lib.call("vc_resample_u8", _p(x), N, H, W, C, 1, H2, _p(b), _p(c), k, _p(y), _stream(x))
        x = y
    return x


_CV_TABLES = {}


def cv2_resize_u8(frames: torch.Tensor, size) -> torch.Tensor:
    """cv2.resize(frame, size) INTER_LINEAR on device uint8 frames [..., H, W, C]; size = (w, h) as
    cv2 takes it (vc_resize_linear_u8; tables from vclip_amd.resize, the host restatement)."""
    from . import resize as R
    w, h = int(size[0]), int(size[1])
    _need(frames.dtype == torch.uint8 and frames.is_cuda and frames.dim() >= 3, "cv2_resize_u8: cuda uint8 [..., H, W, C]")
    x = frames.contiguous()
    H, W, C = x.shape[-3:]
    if (H, W) == (h, w):
        return x.clone()
    N = x.numel() // (H * W * C)
    y = torch.empty(*x.shape[:-3], h, w, C, dtype=torch.uint8, device=x.device)
    area = int(R.is_area_fast_2x((H, W), (h, w)))
    key = (H, W, h, w, x.device)
    if key not in _CV_TABLES:
        xo, xa0, xa1, xlim = R.linear_tables(W, w, clamp=True)
        yo, yb0, yb1, _ = R.linear_tables(H, h, clamp=False)
        tab = np.concatenate([xo, xa0, xa1, yo, yb0, yb1]).astype(np.int32)
        _CV_TABLES[key] = (torch.from_numpy(tab).to(x.device), xlim)
    tab, xlim = _CV_TABLES[key]
    _lib.call("vc_resize_linear_u8", _p(x), N, H, W, C, h, w, _p(tab), xlim, area, _p(y), _stream(x))
    return y


def _transform(frames, idx, T, resize_hw, crop, scale3, shift3, layout, out_bf16=False):
    B, F, H, W, C = frames.shape
    _need(C == 3 and frames.dtype == torch.uint8 and frames.is_contiguous(), "frames: u8 [B, F, H, W, 3]")
    _need(idx.dtype == torch.int64 and idx.is_contiguous() and tuple(idx.shape) == (B, T), "idx: int64 [B, T]")
    rh, rw = resize_hw
    top, left, ch, cw = crop
    shape = (B, T, 3, ch, cw) if layout == 0 else (B, 3, T, ch, cw)
    out = torch.empty(shape, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=frames.device)
    sc = (ctypes.c_float * 3)(*scale3)
    sh = (ctypes.c_float * 3)(*shift3)
    _lib.call("vc_video_transform", _p(frames), B, F, H, W, _p(idx), T, rh, rw, top, left, ch, cw,
              ctypes.addressof(sc), ctypes.addressof(sh), layout, int(out_bf16), _p(out), _stream(frames))
    return out


def vivit_preprocess(frames: torch.Tensor, crop: int = 224, shortest_edge: int = 256) -> torch.Tensor:
    """frames u8 [B, T, H, W, 3] (device) -> pixel_values f32 [B, T, 3, crop, crop]."""
    _dev(frames)
    B, T, H, W, C = frames.shape
    if H <= W:
        nh, nw = shortest_edge, int(shortest_edge * W / H)
    else:
        nh, nw = int(shortest_edge * H / W), shortest_edge
    r = pil_resize_u8(frames.reshape(B * T, H, W, C), (nh, nw)).reshape(B, T, nh, nw, C)
    top, left = (nh - crop) // 2, (nw - crop) // 2
    idx = torch.arange(T, device=frames.device, dtype=torch.int64).repeat(B, 1).contiguous()
    # rescale 1/127.5 with offset -1, then normalise (x - 0.5) / 0.5: net x / 63.75 - 3
    return _transform(r, idx, T, (nh, nw), (top, left, crop, crop), (1 / 63.75,) * 3, (-3.0,) * 3, layout=0)


def uniform_temporal_subsample_indices(num_source: int, num_samples: int) -> torch.Tensor:
    """pytorchvideo UniformTemporalSubsample: torch.linspace(0, t - 1, T).clamp(0, t - 1).long()."""
    return torch.linspace(0, num_source - 1, num_samples).clamp(0, num_source - 1).long()


def short_side_size(h: int, w: int, size: int):
    """pytorchvideo short_side_scale output size."""
    if w < h:
        return int(math.floor((float(h) / w) * size)), size
    return size, int(math.floor((float(w) / h) * size))


def video_eval_transform(frames: torch.Tensor, num_frames: int, short_side: int = 256, crop: int = 224,
                         mean=(0.45, 0.45, 0.45), std=(0.225, 0.225, 0.225), div255: bool = False,
                         layout: str = "bcthw") -> torch.Tensor:
    """frames u8 [B, F, H, W, 3] decoded clip frames (device) -> f32 [B, 3, T, crop, crop]."""
    _dev(frames)
    B, F, H, W, C = frames.shape
    idx = uniform_temporal_subsample_indices(F, num_frames).to(frames.device).repeat(B, 1).contiguous()
    rh, rw = short_side_size(H, W, short_side)
    top, left = int(round((rh - crop) / 2.0)), int(round((rw - crop) / 2.0))
    k = 255.0 if div255 else 1.0
    scale = tuple(1.0 / (k * s) for s in std)
    shift = tuple(-m / s for m, s in zip(mean, std))
    return _transform(frames, idx, num_frames, (rh, rw), (top, left, crop, crop), scale, shift,
                      layout=1 if layout == "bcthw" else 0)


def train_transform_params(n_clips: int, H: int, W: int, min_size: int = 256, max_size: int = 320, crop: int = 224,
                           flip_p: float = 0.5, generator: torch.Generator | None = None):
    """Host draw of the train chain's random parameters, per clip in the reference's order
    (videoswintransformer/swin_video_classifier/data_config/dataset.py:151-163, one clip per
    __getitem__): pytorchvideo RandomShortSideScale `torch.randint(min, max + 1, (1,))`; torchvision
    RandomCrop.get_params `torch.randint(0, h - th + 1, (1,))` then the same for w (no draw when
    the frame already is crop x crop); RandomHorizontalFlip `torch.rand(1) < p`.  torch's default
    generator unless one is given (the reference's DataLoader with num_workers = 0 draws from it).
    Returns int32 [n_clips, 5] {resize_h, resize_w, top, left, flip}."""
    out = []
    for _ in range(n_clips):
        size = int(torch.randint(min_size, max_size + 1, (1,), generator=generator).item())
        rh, rw = short_side_size(H, W, size)
        if rh < crop or rw < crop:
            raise ValueError(f"RandomCrop: required crop {crop} larger than the scaled frame {rh}x{rw}")
        if rh == crop and rw == crop:
            top = left = 0
        else:
            top = int(torch.randint(0, rh - crop + 1, size=(1,), generator=generator).item())
            left = int(torch.randint(0, rw - crop + 1, size=(1,), generator=generator).item())
        flip = int(bool(torch.rand(1, generator=generator) < flip_p))
        out.append((rh, rw, top, left, flip))
    return torch.tensor(out, dtype=torch.int32)


def video_train_transform(frames: torch.Tensor, num_frames: int, min_size: int = 256, max_size: int = 320,
                          crop: int = 224, mean=(0.45, 0.45, 0.45), std=(0.225, 0.225, 0.225), div255: bool = False,
                          layout: str = "bcthw", generator: torch.Generator | None = None, params=None):
    """Train-time chain of the Swin / ResNet3D datasets: frames u8 [B, F, H, W, 3] (device) ->
    f32 [B, 3, T, crop, crop]; UniformTemporalSubsample, RandomShortSideScale(min, max) (torch
    bilinear), RandomCrop(crop), RandomHorizontalFlip, Normalize -- one fused kernel
    (vc_video_transform_clips) with the random parameters drawn on the host
    (`train_transform_params`, or `params` as returned by it).  Returns (clip, params)."""
    _dev(frames)
    B, F, H, W, C = frames.shape
    _need(C == 3 and frames.dtype == torch.uint8 and frames.is_contiguous(), "frames: u8 [B, F, H, W, 3]")
    if params is None:
        params = train_transform_params(B, H, W, min_size, max_size, crop, generator=generator)
    params = params.to(torch.int32).contiguous()
    _need(tuple(params.shape) == (B, 5), "params: int32 [B, 5]")
    for rh, rw, top, left, _ in params.tolist():
        _need(0 <= top and top + crop <= rh and 0 <= left and left + crop <= rw, "crop window outside the frame")
    idx = uniform_temporal_subsample_indices(F, num_frames).to(frames.device).repeat(B, 1).contiguous()
    k = 255.0 if div255 else 1.0
    sc = (ctypes.c_float * 3)(*(1.0 / (k * s) for s in std))
    sh = (ctypes.c_float * 3)(*(-m / s for m, s in zip(mean, std)))
    lay = 1 if layout == "bcthw" else 0
    shape = (B, num_frames, 3, crop, crop) if lay == 0 else (B, 3, num_frames, crop, crop)
    out = torch.empty(shape, dtype=torch.float32, device=frames.device)
    pd = params.to(frames.device)
    _lib.call("vc_video_transform_clips", _p(frames), B, F, H, W, _p(idx), num_frames, _p(pd), crop, crop,
              ctypes.addressof(sc), ctypes.addressof(sh), lay, 0, _p(out), _stream(frames))
    return out, params


def timesformer_preprocess(frames: torch.Tensor, mean=(0.45, 0.45, 0.45), std=(0.225, 0.225, 0.225)) -> torch.Tensor:
    """frames u8 [B, T, 224, 224, 3] -> pixel_values f32 [B, T, 3, 224, 224] = (x/255 - mean)/std."""
    _dev(frames)
    B, T, H, W, C = frames.shape
    idx = torch.arange(T, device=frames.device, dtype=torch.int64).repeat(B, 1).contiguous()
    scale = tuple(1.0 / (255.0 * s) for s in std)
    shift = tuple(-m / s for m, s in zip(mean, std))
    return _transform(frames, idx, T, (H, W), (0, 0, H, W), scale, shift, layout=0)
