"""Shared body of the Swin3D and ResNet3D folders' `VideoDataset` (videoswintransformer/
swin_video_classifier/data_config/dataset.py:18-235, resnet50-3d-video/video_classifier/data_config/
dataset.py:22-243): class folders under `<root_dir>/<mode>`, label = (folder name == 'referral'),
the sampled indices bounding a decoded span `get_clip(idx[0] / fps, (idx[-1] + 1) / fps)`, then the
pytorchvideo transform chain on that span (on the GPU here), item = (clip [1, 3, T, 224, 224],
labels [1])."""
from __future__ import annotations

import logging
import math
from pathlib import Path

import numpy as np
import torch

from .. import video_io


def span_frames(src, start_sec, end_sec):
    """Frames of `src` whose timestamps i / fps lie in [start_sec, end_sec): pytorchvideo
    EncodedVideo.get_clip's half-open window (its PyAV decoder keeps start_pts <= pts < end_pts)."""
    fps = src.fps if src.fps > 0 else 30.0
    lo = max(0, math.ceil(start_sec * fps - 1e-6))
    hi = min(src.total_frames, math.ceil(end_sec * fps - 1e-6))
    if hi <= lo:
        raise ValueError(f"empty clip [{start_sec:.4f}, {end_sec:.4f}) s of {src.path}")
    return src.read(list(range(lo, hi)))


class SpanVideoDataset(torch.utils.data.Dataset):
    def __init__(self, root_dir, mode="train", sampling_method="uniform", num_frames=32, fps=30, stride=0.5,
                 logger=None, device=None):
        self.root_dir = Path(root_dir) / mode
        self.mode = mode
        self.num_frames = num_frames
        self.sampling_method = sampling_method
        self.logger = logger or logging.getLogger(__name__)
        self.fps = fps
        self.stride = stride
        self.device = device

    def _setup_data_paths(self):
        self.video_paths, self.labels = [], []
        for class_path in self.root_dir.iterdir():
            if class_path.is_dir():
                label = 1 if class_path.name == "referral" else 0
                # the reference globs *.mp4; the build also reads its raw .npy clips and frame dirs
                for video_path in video_io.list_videos(class_path):
                    self.video_paths.append(str(video_path))
                    self.labels.append(label)
        self.logger.info(f"Found {len(self.video_paths)} videos for {self.mode} split")
        self.logger.info(f"Class distribution: {sum(self.labels)} referral, "
                         f"{len(self.labels) - sum(self.labels)} non-referral")

    def __len__(self):
        return len(self.video_paths)

    # --- host half of __getitem__ (sampling + decode): runs in DataLoader workers
    def _clip_window(self, src, frame_indices):
        """(start_sec, end_sec) of the decoded span; the folder decides the fps it divides by."""
        raise NotImplementedError

    def load_span(self, idx):
        """(uint8 frames [F, H, W, 3] of the sampled span, label) -- no GPU work."""
        video_path = self.video_paths[idx]
        try:
            src = video_io.open_video(video_path)
            frame_indices = self._indices(video_path, src)
            start_sec, end_sec = self._clip_window(src, frame_indices)
            return np.ascontiguousarray(span_frames(src, start_sec, end_sec)), self.labels[idx]
        except Exception as e:
            self.logger.error(f"Error loading video {video_path}: {str(e)}")
            raise

    # --- device half: UniformTemporalSubsample -> (Random)ShortSideScale -> crop (-> flip) -> Normalize
    def transform_span(self, frames, label):
        from .. import preprocess as pp
        dev = self.device
        if dev is None:
            if not torch.cuda.is_available():
                raise RuntimeError("vclip_amd: the clip transform runs on the GPU (MI355X); no CPU path")
            dev = torch.device("cuda", torch.cuda.current_device())
        fr = torch.from_numpy(np.ascontiguousarray(frames)).to(dev).unsqueeze(0)
        if self.mode == "train":
            clip = pp.video_train_transform(fr, self.num_frames)[0]
        else:
            clip = pp.video_eval_transform(fr, self.num_frames)
        return clip, torch.tensor([label], dtype=torch.long)

    def __getitem__(self, idx):
        if torch.utils.data.get_worker_info() is not None:
            raise RuntimeError("this dataset's transform runs on the GPU, which a DataLoader worker cannot use: "
                               "build the loader with create_dataloaders (workers decode via load_span, the main "
                               "process transforms), or iterate load_span")
        return self.transform_span(*self.load_span(idx))
