"""`videoswintransformer/swin_video_classifier/data_config/` drop-in: `VideoDataset` (dataset.py:18-235),
`video_collate_fn` (dataloader.py:5-19) and `create_dataloaders(args, logger)` (dataloader.py:21-93).

Sampling: global `random` / `numpy` seeded 42 once at construction (dataset.py:41-43), indices and
`dynamic_fps` from vclip_amd.sampling.SwinSampler (bit-exact, tests/golden/sampling.json).  The span
is decoded at the video's own fps (dataset.py:203-214; <= 0 -> 30 with a warning) and clamped to the
video's duration."""
from __future__ import annotations

import random

import numpy as np
import torch

from .. import sampling, video_io
from ._device import DeviceClipLoader
from ._span import SpanVideoDataset

__all__ = ["VideoDataset", "video_collate_fn", "create_dataloaders"]


class VideoDataset(SpanVideoDataset):
    def __init__(self, root_dir, mode="train", sampling_method="uniform", num_frames=32, fps=30, stride=0.5,
                 logger=None, device=None):
        super().__init__(root_dir, mode, sampling_method, num_frames, fps, stride, logger, device)
        random.seed(42)
        np.random.seed(42)
        self._sampler = sampling.SwinSampler(num_frames, sampling_method, self.logger,
                                             fps_of=lambda p: video_io.open_video(p).fps, seed=False)
        self._setup_data_paths()

    def get_sampling_indices(self, video_path, total_frames):
        """(indices, dynamic_fps) -- dataset.py:64-149."""
        return self._sampler.get_sampling_indices(video_path, total_frames)

    def _indices(self, video_path, src):
        return self.get_sampling_indices(video_path, src.total_frames)[0]

    def _clip_window(self, src, frame_indices):
        original_fps = src.fps
        if original_fps <= 0:
            self.logger.warning(f"Invalid FPS value ({original_fps}) for video {src.path}, using default 30 fps")
            original_fps = 30.0
        duration = src.total_frames / original_fps or 10.0
        return max(0, frame_indices[0] / original_fps), min(duration, (frame_indices[-1] + 1) / original_fps)


def video_collate_fn(batch):
    """(clips [B, min_clips, C, T, H, W], labels [B, min_clips]) -- dataloader.py:5-19."""
    min_clips = min(sample_clips.size(0) for sample_clips, _ in batch)
    clips = torch.stack([c[:min_clips] for c, _ in batch], dim=0)
    labels = torch.stack([lab[:min_clips] for _, lab in batch], dim=0)
    return clips, labels


def create_dataloaders(args, logger):
    """{'train', 'val', 'test'} loaders; args: data_dir, test_data_dir, {train,val,test}_sampling,
    num_frames, batch_size, num_workers (dataloader.py:21-93)."""
    sampling_methods = {"train": args.train_sampling, "val": args.val_sampling, "test": args.test_sampling}
    logger.info("Creating datasets with the following sampling methods:")
    for split, method in sampling_methods.items():
        logger.info(f"{split}: {method}")
    dataloaders = {}
    for split in ("train", "val", "test"):
        root = (args.test_data_dir or args.data_dir) if split == "test" else args.data_dir
        try:
            ds = VideoDataset(root, mode=split, sampling_method=sampling_methods[split], num_frames=args.num_frames,
                              logger=logger)
            dataloaders[split] = DeviceClipLoader(ds, batch_size=args.batch_size, shuffle=(split == "train"),
                                                  num_workers=args.num_workers, collate_fn=video_collate_fn)
            logger.info(f"Created {split} dataloader with {len(dataloaders[split])} batches (batch size: "
                        f"{args.batch_size})")
        except Exception as e:
            logger.error(f"Error creating {split} dataset/dataloader: {str(e)}")
            raise
    return dataloaders
