"""`VideoDataset` — drop-in for the ViViT / TimeSformer folders' dataset class.

Same constructor, attributes and item dict as
`vivit_transformer/vivit_classifier/data_config/dataset.py:10-381` (the TimeSformer folder's
`data_config/dataset.py` is the same class):

  VideoDataset(root_dir, mode='train', sampling_method='uniform', num_frames=32, logger=None)
    .data_dir / .mode / .num_frames / .sampling_method / .video_paths / .labels / .class_labels
    ._verify_video_integrity(p) / ._load_dataset() / .get_video_properties(p)
    .get_sampling_indices(video_path, total_frames) -> list[int]      (dataset.py:129-193)
    len(ds), ds[i] -> {'pixel_values': uint8 [T, 224, 224, 3], 'labels': tensor(label),
                       'video_path': str, 'frame_indices': list[int]}  (dataset.py:198-292)

* Directory fallback of dataset.py:23-31 (`<root>/dataset/<mode>`, `<root>/<mode>`).
* Seeds `random` and `numpy` with 42 once at construction (dataset.py:39-40) and draws indices
  from the global `random` stream in `__getitem__` call order, so the indices are bit-exact with
  the reference for the same call sequence (tests/test_video_dataset.py replays
  tests/golden/sampling.json, generated from the reference sampler itself).
* Class folders are walked in `Path.iterdir()` order and videos in `glob` order, as the reference
  does; labels index the sorted class names.  Besides `*.mp4` the build accepts its raw clip format
  (`*.npy`, uint8 [F, H, W, 3]) and frame directories (video_io.py), since PyAV / OpenCV are absent
  here.
* Frames are gathered at the sampled indices (clamped, as dataset.py:250-251), padded / trimmed to
  `num_frames`, and resized to 224x224 with OpenCV's INTER_LINEAR restated in resize.py when the
  source is another size (dataset.py:271-277).
* Errors: an unreadable video yields the reference's gray placeholder (127) with empty
  `frame_indices` and a warning (dataset.py:371-381); the reference's intermediate PyAV -> OpenCV
  retry has no counterpart (one decoder per format here).
"""
from __future__ import annotations

import logging
import random
from pathlib import Path

import numpy as np
import torch

from .resize import resize_linear_u8
from .sampling import sample_indices
from .video_io import open_video

_EXTRA_PATTERNS = ("*.npy",)


class VideoDataset(torch.utils.data.Dataset):
    def __init__(self, root_dir, mode="train", sampling_method="uniform", num_frames=32, logger=None):
        self.root_dir = Path(root_dir)
        if not (self.root_dir / "dataset").exists():
            if (self.root_dir / mode).exists():
                self.data_dir = self.root_dir / mode
            else:
                self.root_dir = self.root_dir / "dataset"
                self.data_dir = self.root_dir / mode
        else:
            self.data_dir = self.root_dir / "dataset" / mode
        self.mode = mode
        self.num_frames = num_frames
        self.sampling_method = sampling_method
        self.logger = logger or logging.getLogger(__name__)
        random.seed(42)
        np.random.seed(42)
        self.video_paths = []
        self.labels = []
        self.class_labels = []
        self._load_dataset()

    def _verify_video_integrity(self, video_path) -> bool:
        try:
            src = open_video(video_path)
            if src.total_frames <= 0:
                self.logger.warning(f"Video {video_path} has no frames")
                return False
            src.read([0])
            return True
        except Exception as e:  # noqa: BLE001 - the reference logs and skips any failure
            self.logger.warning(f"Error verifying video {video_path}: {str(e)}")
            return False

    def _videos_of(self, class_dir: Path) -> list:
        files = list(class_dir.glob("*.mp4"))
        for pat in _EXTRA_PATTERNS:
            files += list(class_dir.glob(pat))
        files += [d for d in class_dir.iterdir() if d.is_dir()]
        return files

    def _load_dataset(self):
        if not self.data_dir.exists():
            raise FileNotFoundError(f"Data directory not found: {self.data_dir}")
        class_dirs = [d for d in self.data_dir.iterdir() if d.is_dir()]
        self.class_labels = sorted([d.name for d in class_dirs])
        self.logger.info(f"Found {len(class_dirs)} classes: {self.class_labels}")
        label_map = {label: idx for idx, label in enumerate(self.class_labels)}
        for class_dir in class_dirs:
            label_idx = label_map[class_dir.name]
            video_files = self._videos_of(class_dir)
            if not video_files:
                self.logger.warning(f"No .mp4 files found in {class_dir}")
            valid = [p for p in video_files if self._verify_video_integrity(p)]
            if len(video_files) - len(valid) > 0:
                self.logger.warning(f"Skipped {len(video_files) - len(valid)} invalid videos in class '{class_dir.name}'")
            self.logger.info(f"Found {len(valid)} valid videos in class '{class_dir.name}'")
            for p in valid:
                self.video_paths.append(p)
                self.labels.append(label_idx)
        self.logger.info(f"Total videos for {self.mode}: {len(self.video_paths)} using {self.sampling_method} sampling")

    def get_video_properties(self, video_path):
        """(total_frames, fps, duration_sec, width, height), dataset.py:114-127."""
        src = open_video(video_path)
        first = src.read([0])
        total, fps = src.total_frames, src.fps
        return total, fps, total / fps, int(first.shape[2]), int(first.shape[1])

    def get_sampling_indices(self, video_path, total_frames):
        if total_frames < self.num_frames:
            self.logger.info(f"Video has {total_frames} frames, which is less than the requested "
                             f"{self.num_frames} frames.")
        return sample_indices(total_frames, self.num_frames, self.sampling_method)

    def __len__(self):
        return len(self.video_paths)

    def _placeholder(self, label, video_path):
        return {"pixel_values": np.ones((self.num_frames, 224, 224, 3), dtype=np.uint8) * 127,
                "labels": torch.tensor(label), "video_path": str(video_path), "frame_indices": []}

    def __getitem__(self, idx):
        video_path = self.video_paths[idx]
        label = self.labels[idx]
        try:
            src = open_video(video_path)
            total_frames, fps = src.total_frames, src.fps
            if total_frames == 0 or fps <= 0:
                raise ValueError(f"Invalid video: {video_path} - no frames or zero duration")
            frame_indices = self.get_sampling_indices(video_path, total_frames)
            frames = list(src.read(frame_indices))
            frames = frames[: self.num_frames]
            while len(frames) < self.num_frames:
                frames.append(frames[-1])
            video_array = np.stack(frames)
            if video_array.shape[1:3] != (224, 224):
                video_array = resize_linear_u8(video_array, (224, 224))
            return {"pixel_values": video_array.astype(np.uint8, copy=False), "labels": torch.tensor(label),
                    "video_path": str(video_path), "frame_indices": frame_indices}
        except Exception as e:  # noqa: BLE001 - reference: log, return a placeholder
            self.logger.warning(f"Failed to load {video_path}: {str(e)}; returning a placeholder")
            return self._placeholder(label, video_path)
