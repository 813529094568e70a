"""Host-side frame sampling API — drop-in for the reference samplers, bit-exact.

Sampling stays on the host in Python (SURVEY.md §7 "Hard parts"): its cost is µs per
clip and bit-exactness depends on CPython's MT19937 stream consumed through exactly
the same `random` calls (`sample`, `randint`, `choices`, `random`) in the same order.
Only the frame gather that consumes these indices runs on the GPU
(`vclip_amd.ops.frame_gather`).

One core (`sample_indices`) restates the shared algorithm of
`vivit_transformer/vivit_classifier/data_config/dataset.py:129-193` (identical in
`timesformer/timesformer_classifier/data_config/dataset.py:137-201`); thin wrappers
reproduce every folder's seeding/caching/return-type quirks:

* ViViT / TimeSformer dataset: global `random` seeded 42 once at construction.
* Swin dataset: returns `(indices, dynamic_fps)`; short videos read fps (≤0 -> 30).
  `videoswintransformer/swin_video_classifier/data_config/dataset.py:64-149`
* Swin inference: module function reseeding 42 on every call.
  `videoswintransformer/inference.py:94-185`
* ResNet3D dataset: per-video seed `hash(basename) % 10_000_000`, cached, then global
  reseed 42 (random, numpy, torch).  `resnet50-3d-video/video_classifier/data_config/dataset.py:79-169`
* ResNet3D inference: same, returns `(indices, dynamic_fps)`.  `resnet50-3d-video/inference.py:90-185`
* ResNet50-LSTM dataset: `random.seed(42)` on every call.  `resnet50-2d-lstm/src/data_config/dataset.py:85-163`
* ResNet50-LSTM inference: numpy RNG samplers clamping T to total.  `resnet50-2d-lstm/inference.py:74-130`
* `data_handling.sample_frame_indices`: contiguous window via numpy.  `data_handling.py:41-56`
"""
from __future__ import annotations

import logging
import math
import os
import random
from typing import Callable, Optional

import numpy as np

SAMPLING_METHODS = ("random", "uniform", "random_window")  # CLI choices, vivit_transformer/main.py:28-36


def _default_fps(video_path: str) -> float:
    """fps of a video file (reference: cv2.CAP_PROP_FPS).  cv2 is optional on this image."""
    try:
        import cv2  # type: ignore
    except ImportError as e:  # pragma: no cover - exercised only without a decoder
        raise RuntimeError(
            f"short-video sampling for {video_path} needs the source fps; cv2 is not installed — "
            "pass fps_of=<callable> to the sampler") from e
    cap = cv2.VideoCapture(str(video_path))
    fps = cap.get(cv2.CAP_PROP_FPS)
    cap.release()
    return fps


def sample_indices(total_frames: int, num_frames: int, method: str, rng=random) -> list:
    """Frame indices for one clip.  `rng` is the `random` module (global stream, as the
    reference uses) or a `random.Random` instance.  dataset.py:129-193."""
    T = num_frames
    if total_frames >= T:
        if method == "random":
            return sorted(rng.sample(range(total_frames), T))
        if method == "random_window":
            w = total_frames / T
            out = []
            for i in range(T):
                start = int(i * w)
                end = min(int((i + 1) * w), total_frames)
                end = max(end, start + 1)
                out.append(rng.randint(start, end - 1))
            return out
        if T == 1:
            return [total_frames // 2]
        step = (total_frames - 1) / (T - 1)
        return [min(int(i * step), total_frames - 1) for i in range(T)]
    # fewer frames than requested: duplicates allowed
    if method == "random":
        return sorted(rng.choices(range(total_frames), k=T))
    if method == "random_window":
        w = total_frames / T
        out = []
        for i in range(T):
            vs = i * w
            ve = (i + 1) * w
            out.append(min(int(math.floor(vs + (ve - vs) * rng.random())), total_frames - 1))
        return out
    if T == 1:
        return [total_frames // 2]
    step = total_frames / T
    return [min(int(i * step), total_frames - 1) for i in range(T)]


class _Base:
    def __init__(self, num_frames: int = 32, sampling_method: str = "uniform", logger=None):
        self.num_frames = num_frames
        self.sampling_method = sampling_method
        self.logger = logger or logging.getLogger(__name__)


class VivitSampler(_Base):
    """`VideoDataset.get_sampling_indices` of the ViViT / TimeSformer folders.
    Construction seeds the global streams exactly like `VideoDataset.__init__`
    (vivit dataset.py:38-40; timesformer dataset.py:46-47)."""

    def __init__(self, num_frames: int = 32, sampling_method: str = "uniform", logger=None, seed: bool = True):
        super().__init__(num_frames, sampling_method, logger)
        if seed:
            random.seed(42)
            np.random.seed(42)

    def get_sampling_indices(self, video_path, total_frames: int) -> list:
        if total_frames < self.num_frames:
            self.logger.info(f"Video has {total_frames} frames, which is less than the requested "
                             f"{self.num_frames} frames.")
        return sample_indices(total_frames, self.num_frames, self.sampling_method)


TimesformerSampler = VivitSampler


class SwinSampler(_Base):
    """Swin dataset sampler: returns `(indices, dynamic_fps)` (swin dataset.py:64-149)."""

    def __init__(self, num_frames: int = 32, sampling_method: str = "uniform", logger=None,
                 fps_of: Optional[Callable[[str], float]] = None, seed: bool = True):
        super().__init__(num_frames, sampling_method, logger)
        self.fps_of = fps_of or _default_fps
        if seed:
            random.seed(42)
            np.random.seed(42)

    def get_sampling_indices(self, video_path, total_frames: int):
        dynamic_fps = None
        if total_frames < self.num_frames:
            fps = self.fps_of(str(video_path))
            if fps <= 0:
                self.logger.warning(f"Invalid FPS value ({fps}) for video {video_path}, using default 30 fps")
                fps = 30.0
            dynamic_fps = self.num_frames / (total_frames / fps)
        return sample_indices(total_frames, self.num_frames, self.sampling_method), dynamic_fps


def swin_inference_sampling_indices(video_path, total_frames, num_frames, sampling_method, logger=None,
                                    fps_of: Optional[Callable[[str], float]] = None):
    """Module-level sampler of videoswintransformer/inference.py:94-185 (reseeds 42 every call)."""
    random.seed(42)
    np.random.seed(42)
    dynamic_fps = None
    if total_frames < num_frames:
        fps = (fps_of or _default_fps)(str(video_path))
        if fps <= 0:
            fps = 30.0
        dynamic_fps = num_frames / (total_frames / fps)
    return sample_indices(total_frames, num_frames, sampling_method), dynamic_fps


def _reseed_all(seed: int):
    random.seed(seed)
    np.random.seed(seed)
    try:
        import torch
        torch.manual_seed(seed)
    except ImportError:  # pragma: no cover
        pass


class Resnet3dSampler(_Base):
    """ResNet3D dataset sampler (resnet50-3d-video dataset.py:79-169): per-video seed
    `hash(basename) % 10_000_000` (depends on PYTHONHASHSEED, as in the reference),
    cached per path, global streams reset to 42 afterwards.  Returns a list."""

    def __init__(self, num_frames: int = 32, sampling_method: str = "uniform", logger=None,
                 fps_of: Optional[Callable[[str], float]] = None, seed: bool = True):
        super().__init__(num_frames, sampling_method, logger)
        self.fps_of = fps_of or _default_fps
        self.cached_indices = {}
        if seed:
            _reseed_all(42)

    def _fresh(self, video_path, total_frames):
        video_seed = int(hash(os.path.basename(video_path)) % 10000000)
        random.seed(video_seed)
        np.random.seed(video_seed)
        dynamic_fps = None
        if total_frames < self.num_frames:
            fps = self.fps_of(str(video_path))  # no <=0 guard in the reference (ZeroDivisionError)
            dynamic_fps = self.num_frames / (total_frames / fps)
        idx = sample_indices(total_frames, self.num_frames, self.sampling_method)
        _reseed_all(42)
        return idx, dynamic_fps

    def get_sampling_indices(self, video_path, total_frames: int) -> list:
        if video_path in self.cached_indices:
            return self.cached_indices[video_path]
        idx, _ = self._fresh(video_path, total_frames)
        self.cached_indices[video_path] = idx
        return idx


class Resnet3dInferenceSampler(Resnet3dSampler):
    """`VideoInference.get_sampling_indices` (resnet50-3d-video/inference.py:90-185):
    like the dataset sampler but returns `(indices, dynamic_fps)`; fps cached only when truthy."""

    def __init__(self, num_frames: int = 32, sampling_method: str = "uniform", logger=None,
                 fps_of: Optional[Callable[[str], float]] = None):
        super().__init__(num_frames, sampling_method, logger, fps_of, seed=False)
        self.sampled_frames = {}
        self.dynamic_fps_info = {}

    def get_sampling_indices(self, video_path, total_frames: int):
        if video_path in self.sampled_frames:
            return self.sampled_frames[video_path], self.dynamic_fps_info.get(video_path)
        idx, dfps = self._fresh(video_path, total_frames)
        self.sampled_frames[video_path] = idx
        if dfps:
            self.dynamic_fps_info[video_path] = dfps
        return idx, dfps


class LstmSampler(_Base):
    """ResNet50-LSTM dataset sampler: `random.seed(42)` on every call
    (resnet50-2d-lstm/src/data_config/dataset.py:85-163)."""

    def __init__(self, sequence_length: int = 32, sampling_method: str = "uniform", logger=None):
        super().__init__(sequence_length, sampling_method, logger)
        self.sequence_length = sequence_length

    def get_sampling_indices(self, video_path, total_frames: int) -> list:
        random.seed(42)
        return sample_indices(total_frames, self.sequence_length, self.sampling_method)


# ---- resnet50-2d-lstm/inference.py:74-130: numpy-RNG samplers (T clamped to total) ----
def lstm_random_sampling(total_frames: int, num_frames: int) -> list:
    np.random.seed(42)
    num_frames = min(num_frames, total_frames)
    return sorted(np.random.choice(total_frames, num_frames, replace=False))


def lstm_uniform_sampling(total_frames: int, num_frames: int) -> list:
    num_frames = min(num_frames, total_frames)
    if num_frames == 1:
        return [total_frames // 2]
    step = (total_frames - 1) / (num_frames - 1)
    return [min(int(i * step), total_frames - 1) for i in range(num_frames)]


def lstm_random_window_sampling(total_frames: int, num_frames: int) -> list:
    np.random.seed(42)
    num_frames = min(num_frames, total_frames)
    w = total_frames / num_frames
    out = []
    for i in range(num_frames):
        start = int(i * w)
        end = max(min(int((i + 1) * w), total_frames), start + 1)
        out.append(np.random.randint(start, end))
    return out


# ---- data_handling.py:41-56 ----
def sample_frame_indices(clip_len, frame_sample_rate, seg_len):
    """Contiguous clip of `clip_len` indices ending at a random point (numpy global RNG)."""
    converted_len = int(clip_len * frame_sample_rate)
    end_idx = np.random.randint(converted_len, seg_len)
    start_idx = end_idx - converted_len
    indices = np.linspace(start_idx, end_idx, num=clip_len)
    return np.clip(indices, start_idx, end_idx - 1).astype(np.int64)
