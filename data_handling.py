"""`data_handling` drop-in: the reference's top-level helper module (`/data_handling.py`), importable
as `import data_handling` from the repository root, same function names and return types.

  generate_all_files(root, only_files=True)                 data_handling.py:7-11
  read_video_pyav(container, indices) -> uint8 [n, 224, 224, 3]   :12-38
  sample_frame_indices(clip_len, frame_sample_rate, seg_len) -> int64 [clip_len]   :41-56
  frames_convert_and_create_dataset_dictionary(directory, number_of_frames=10)   :59-113

`sample_frame_indices` is the bit-exact sampler of vclip_amd.sampling (numpy global RNG, pinned to
tests/golden/sampling.json).  PyAV is not in this image: `read_video_pyav` decodes a PyAV container
exactly as the reference when PyAV is installed, and otherwise accepts the build's video sources
(a path to a raw `.npy` clip or a frame directory, or a vclip_amd.video_io.VideoSource); frames are
scaled to 224x224 with OpenCV's INTER_LINEAR restatement (vclip_amd/resize.py) where the reference
uses PyAV's `frame.reformat` (swscale bilinear): parity unpinned for non-224 sources.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import vclip_amd  # noqa: E402,F401  (registers the package)
from vclip_amd.resize import resize_linear_u8  # noqa: E402
from vclip_amd.sampling import sample_frame_indices  # noqa: E402,F401
from vclip_amd.video_io import VideoSource, open_video  # noqa: E402

__all__ = ["generate_all_files", "read_video_pyav", "sample_frame_indices",
           "frames_convert_and_create_dataset_dictionary"]


def generate_all_files(root: Path, only_files: bool = True):
    for p in Path(root).rglob("*"):
        if only_files and not p.is_file():
            continue
        yield p


def read_video_pyav(container, indices):
    """Frames whose decode position is in `indices` (once each, in stream order, from indices[0]
    to indices[-1]), 224x224 RGB uint8.  Raises ValueError when none is extracted."""
    start_index, end_index = int(indices[0]), int(indices[-1])
    print(f"Reading frames from {start_index} to {end_index}")
    wanted = set(int(i) for i in indices)
    if hasattr(container, "decode"):  # a PyAV container (PyAV installed)
        container.seek(0)
        frames = []
        for i, frame in enumerate(container.decode(video=0)):
            if i > end_index:
                break
            if i >= start_index and i in wanted:
                frames.append(frame.reformat(width=224, height=224))
        print(f"Number of frames extracted: {len(frames)}")
        if len(frames) == 0:
            raise ValueError("No frames were extracted!")
        new = np.stack([x.to_ndarray(format="rgb24") for x in frames])
    else:
        src = container if isinstance(container, VideoSource) else open_video(container)
        keep = [i for i in sorted(wanted) if start_index <= i <= end_index and i < src.total_frames]
        print(f"Number of frames extracted: {len(keep)}")
        if len(keep) == 0:
            raise ValueError("No frames were extracted!")
        new = src.read(keep)
        if new.shape[1:3] != (224, 224):
            new = resize_linear_u8(new, (224, 224))
    print(f"Final video array shape: {new.shape}")
    return new


def _open_container(path):
    try:
        import av  # noqa: F401
        return av.open(str(path))
    except ImportError:
        return open_video(path)


def frames_convert_and_create_dataset_dictionary(directory, number_of_frames=10):
    class_labels = []
    all_videos = []
    sizes = []
    dir_path = Path(directory)
    for split in ["train", "test", "val"]:
        split_path = dir_path / "dataset" / split
        if not split_path.exists():
            continue
        for class_path in split_path.iterdir():
            if not class_path.is_dir():
                continue
            cls = class_path.name
            if cls not in class_labels:
                class_labels.append(cls)
            for video_file in list(class_path.glob("*.mp4")) + list(class_path.glob("*.npy")):
                container = None
                try:
                    container = _open_container(video_file)
                    num_frames = (container.streams.video[0].frames if hasattr(container, "streams")
                                  else container.total_frames)
                    print(f"Processing file {video_file} number of Frames: {num_frames}")
                    indices = sample_frame_indices(clip_len=number_of_frames, frame_sample_rate=1, seg_len=num_frames)
                    video = read_video_pyav(container=container, indices=indices)
                    all_videos.append({"video": video, "labels": cls, "split": split, "path": str(video_file)})
                    sizes.append(num_frames)
                except Exception as e:  # noqa: BLE001 - the reference prints and continues
                    print(f"Error processing {video_file}: {str(e)}")
                finally:
                    if container is not None and hasattr(container, "close"):
                        container.close()
    sizes = np.array(sizes)
    print(f"Min number frames {sizes.min()}")
    return all_videos, class_labels
