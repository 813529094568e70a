"""`timesformer/timesformer_classifier/data_config/` drop-in.  Its dataset is the ViViT folder's class
plus an `inference` mode (dataset.py:24-28, 204-216: `root_dir` is the video itself, one item, label
0); its test loader uses `video_collate_fn` too (dataloader.py:122-123)."""
from __future__ import annotations

from pathlib import Path

from ..video_dataset import VideoDataset as _VivitDataset
from .vivit import _create, video_collate_fn

__all__ = ["VideoDataset", "video_collate_fn", "create_dataloaders"]


class VideoDataset(_VivitDataset):
    def __init__(self, root_dir, mode="train", sampling_method="uniform", num_frames=32, logger=None):
        self.is_inference = mode == "inference"
        if self.is_inference:
            import logging
            import random

            import numpy as np
            self.root_dir = self.data_dir = Path(root_dir)
            self.mode, self.num_frames, self.sampling_method = mode, num_frames, sampling_method
            self.logger = logger or logging.getLogger(__name__)
            random.seed(42)
            np.random.seed(42)
            self.video_paths, self.labels, self.class_labels = [self.root_dir], [0], []
        else:
            super().__init__(root_dir, mode, sampling_method, num_frames, logger)

    def __len__(self):
        return 1 if self.is_inference else super().__len__()


def create_dataloaders(args, sampling_methods, logger):
    return _create(VideoDataset, args, sampling_methods, logger, test_collate=True)
