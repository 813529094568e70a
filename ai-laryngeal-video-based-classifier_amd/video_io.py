"""Host video access for the CLIs: frame count, fps and the frames at sampled indices.

The reference decodes with PyAV / pytorchvideo `EncodedVideo` and falls back to OpenCV
(vivit_transformer/vivit_classifier/data_config/dataset.py:198-292, 316-358;
vivit_transformer/inference.py:143-157: per-index `cap.set(POS_FRAMES)`, BGR->RGB).  Neither
library is in this image, so backends are chosen per file:

  * `.npy`           uint8 [F, H, W, 3] RGB, memory-mapped (the build's raw clip format, used by
                     the tests and for pre-decoded datasets); fps from a sibling `<stem>.fps` file
                     or 30;
  * a directory      of image files (`*.png` / `*.jpg`, sorted by name) read with Pillow;
  * `.mp4` / other   PyAV if importable, else OpenCV if importable, else a clear error.

Every backend returns RGB uint8 [T, H, W, 3] for a list of indices (clamped to [0, F-1] like
dataset.py:252-253).  Decoding is host work; the sampled frames then go to the GPU.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np

VIDEO_EXTS = (".mp4", ".avi", ".mov", ".mkv", ".npy")


class VideoSource:
    def __init__(self, path):
        self.path = Path(path)
        self.total_frames = 0
        self.fps = 30.0

    def read(self, indices) -> np.ndarray:
        raise NotImplementedError


class NpyVideo(VideoSource):
    def __init__(self, path):
        super().__init__(path)
        self.frames = np.load(str(path), mmap_mode="r")
        if self.frames.dtype != np.uint8 or self.frames.ndim != 4 or self.frames.shape[-1] != 3:
            raise ValueError(f"{path}: expected uint8 [F, H, W, 3], got {self.frames.dtype} {self.frames.shape}")
        self.total_frames = int(self.frames.shape[0])
        fps_file = self.path.with_suffix(".fps")
        if fps_file.exists():
            self.fps = float(fps_file.read_text().strip())

    def read(self, indices):
        idx = np.clip(np.asarray(indices, dtype=np.int64), 0, self.total_frames - 1)
        return np.ascontiguousarray(self.frames[idx])


class FrameDirVideo(VideoSource):
    def __init__(self, path):
        super().__init__(path)
        self.files = sorted(p for p in self.path.iterdir() if p.suffix.lower() in (".png", ".jpg", ".jpeg"))
        self.total_frames = len(self.files)

    def read(self, indices):
        from PIL import Image
        idx = np.clip(np.asarray(indices, dtype=np.int64), 0, self.total_frames - 1)
        return np.stack([np.asarray(Image.open(self.files[i]).convert("RGB")) for i in idx])


class PyAVVideo(VideoSource):
    def __init__(self, path):
        import av  # noqa: F401  (absent in this image; used when installed)
        super().__init__(path)
        with av.open(str(path)) as c:
            s = c.streams.video[0]
            self.total_frames = int(s.frames)
            self.fps = float(s.average_rate) if s.average_rate else 30.0

    def read(self, indices):
        import av
        idx = np.clip(np.asarray(indices, dtype=np.int64), 0, self.total_frames - 1)
        want = set(int(i) for i in idx)
        got = {}
        with av.open(str(self.path)) as c:
            for i, fr in enumerate(c.decode(video=0)):
                if i in want:
                    got[i] = fr.to_ndarray(format="rgb24")
                if i >= max(want):
                    break
        last = got[max(got)] if got else None
        return np.stack([got.get(int(i), last) for i in idx])


class OpenCVVideo(VideoSource):
    def __init__(self, path):
        import cv2  # noqa: F401  (absent in this image; used when installed)
        super().__init__(path)
        cap = cv2.VideoCapture(str(path))
        if not cap.isOpened():
            raise ValueError(f"Could not open video: {path}")
        self.total_frames = int(cap.get(cv2.CAP_PROP_FRAME_COUNT))
        self.fps = cap.get(cv2.CAP_PROP_FPS) or 30.0
        cap.release()

    def read(self, indices):
        import cv2
        cap = cv2.VideoCapture(str(self.path))
        out = []
        for i in np.clip(np.asarray(indices, dtype=np.int64), 0, self.total_frames - 1):
            cap.set(cv2.CAP_PROP_POS_FRAMES, int(i))  # inference.py:143-152
            ok, fr = cap.read()
            if not ok:
                fr = out[-1][..., ::-1] if out else np.zeros((224, 224, 3), np.uint8)
            out.append(cv2.cvtColor(fr, cv2.COLOR_BGR2RGB))
        cap.release()
        return np.stack(out)


def open_video(path) -> VideoSource:
    p = Path(path)
    if p.is_dir():
        return FrameDirVideo(p)
    if p.suffix.lower() == ".npy":
        return NpyVideo(p)
    errs = []
    for cls in (PyAVVideo, OpenCVVideo):
        try:
            return cls(p)
        except ImportError as e:
            errs.append(str(e))
    raise RuntimeError(f"cannot decode {path}: neither PyAV nor OpenCV is installed ({'; '.join(errs)}); "
                       "decode the clip to a uint8 [F,H,W,3] .npy (or a directory of frames) instead")


def list_videos(class_dir) -> list:
    """Videos of one class folder, as the reference globs `*.mp4` (dataset.py:91) plus the
    build's raw `.npy` clips and frame directories."""
    d = Path(class_dir)
    out = []
    for p in sorted(d.iterdir()):
        if p.is_dir() or p.suffix.lower() in VIDEO_EXTS:
            out.append(p)
    return out


def exists(path) -> bool:
    return os.path.exists(path)
