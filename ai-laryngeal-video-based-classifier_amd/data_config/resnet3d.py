"""`resnet50-3d-video/video_classifier/data_config/` drop-in: `VideoDataset` (dataset.py:22-289),
`video_collate_fn` (dataloader.py:5-19) and `create_dataloaders(args, logger, log_dir=None)`
(dataloader.py:21-101, returns (datasets, dataloaders)).

Sampling: per-video seed `hash(basename) % 10_000_000`, indices cached per path, then random / numpy /
torch reseeded 42 (vclip_amd.sampling.Resnet3dSampler, bit-exact under the same PYTHONHASHSEED).  The
span window divides by the dataset's constant `fps` (30), not the video's (dataset.py:219-222), and is
decoded at the video's real frame rate.  `save_sampled_indices` writes the reference's only golden
artefact, `<log_dir>/sampled_frames_<mode>_<method>.csv` (dataset.py:245-289).  The test and train
loaders use torch's default collate, as the reference passes none."""
from __future__ import annotations

import csv
import os

from .. import sampling, video_io
from ._device import DeviceClipLoader
from ._span import SpanVideoDataset
from .swin import video_collate_fn

__all__ = ["VideoDataset", "video_collate_fn", "create_dataloaders"]


class VideoDataset(SpanVideoDataset):
    def __init__(self, root_dir, mode="train", sampling_method="uniform", num_frames=32, fps=30, stride=0.5,
                 logger=None, log_dir=None, device=None):
        super().__init__(root_dir, mode, sampling_method, num_frames, fps, stride, logger, device)
        self.log_dir = log_dir
        self._sampler = sampling.Resnet3dSampler(num_frames, sampling_method, self.logger,
                                                 fps_of=lambda p: video_io.open_video(p).fps, seed=False)
        self.cached_indices = self._sampler.cached_indices
        self.set_random_seed(42)
        self._setup_data_paths()

    def set_random_seed(self, seed):
        sampling._reseed_all(seed)

    def get_sampling_indices(self, video_path, total_frames):
        """list of indices, cached per path -- dataset.py:79-169."""
        return self._sampler.get_sampling_indices(video_path, total_frames)

    def _indices(self, video_path, src):
        return self.get_sampling_indices(video_path, src.total_frames)

    def _clip_window(self, src, frame_indices):
        duration = (src.total_frames / src.fps if src.fps > 0 else 0.0) or 10.0
        return max(0, frame_indices[0] / self.fps), min(duration, (frame_indices[-1] + 1) / self.fps)

    def save_sampled_indices(self):
        """`<log_dir>/sampled_frames_<mode>_<method>.csv`: video_filename, total_frames, comma-joined
        indices, rows in sorted path order (dataset.py:245-289)."""
        if not self.log_dir:
            self.logger.warning("No log directory provided, cannot save sampled indices")
            return None
        totals = {}
        for video_path in self.video_paths:
            totals[video_path] = video_io.open_video(video_path).total_frames
            if video_path not in self.cached_indices:
                self.get_sampling_indices(video_path, totals[video_path])
        csv_path = os.path.join(self.log_dir, f"sampled_frames_{self.mode}_{self.sampling_method}.csv")
        with open(csv_path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["video_filename", "total_frames", "sampled_frames"])
            for video_path in sorted(self.video_paths):
                w.writerow([os.path.basename(video_path), totals[video_path],
                            ",".join(map(str, self.cached_indices[video_path]))])
        self.logger.info(f"Saved {len(self.cached_indices)} sampled frame records to {csv_path}")
        return csv_path


def create_dataloaders(args, logger, log_dir=None):
    sampling_methods = {"train": args.train_sampling, "val": args.val_sampling, "test": args.test_sampling}
    logger.info("Creating datasets with the following sampling methods:")
    for split, method in sampling_methods.items():
        logger.info(f"{split}: {method}")
    datasets, dataloaders = {}, {}
    for split in ("train", "val", "test"):
        root = (args.test_data_dir or args.data_dir) if split == "test" else args.data_dir
        try:
            datasets[split] = VideoDataset(root, mode=split, sampling_method=sampling_methods[split],
                                           num_frames=args.num_frames, logger=logger, log_dir=log_dir)
            if log_dir:
                datasets[split].save_sampled_indices()
            dataloaders[split] = DeviceClipLoader(datasets[split], batch_size=args.batch_size,
                                                  shuffle=(split == "train"), num_workers=args.num_workers)
            logger.info(f"Created {split} dataloader with {len(dataloaders[split])} batches (batch size: "
                        f"{args.batch_size})")
        except Exception as e:
            logger.error(f"Error creating {split} dataset/dataloader: {str(e)}")
            raise
    return datasets, dataloaders
