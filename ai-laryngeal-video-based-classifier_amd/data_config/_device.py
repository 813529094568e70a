"""Host decode in DataLoader workers, clip transform on the GPU in the main process."""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, Dataset


def _as_batch(items):
    return items


class _HostSpans(Dataset):
    """The host half of a Swin3D / ResNet3D `__getitem__` (sampling + decode), safe in a worker."""

    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, idx):
        return self.ds.load_span(idx)


class DeviceClipLoader:
    """Iterable with the reference DataLoader's batches for the Swin3D / ResNet3D datasets.

    A torch DataLoader over `_HostSpans(dataset)` (batch_size, shuffle, num_workers as given; the
    workers decode) yields lists of (uint8 frames [F, H, W, 3], label); each clip is transformed on
    the GPU by `dataset.transform_span` and the batch is collated by `collate` (the folder's
    `video_collate_fn`, or torch's default collate where the reference passes none)."""

    def __init__(self, dataset, batch_size=1, shuffle=False, num_workers=0, collate_fn=None, pin_memory=False):
        self.dataset = dataset
        self.batch_size = batch_size
        self.num_workers = num_workers
        self.collate_fn = collate_fn or torch.utils.data.default_collate
        self.loader = DataLoader(_HostSpans(dataset), batch_size=batch_size, shuffle=shuffle,
                                 num_workers=num_workers, collate_fn=_as_batch)

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for items in self.loader:
            yield self.collate_fn([self.dataset.transform_span(frames, label) for frames, label in items])
