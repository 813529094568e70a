"""Per-folder dataset / DataLoader drop-ins (vclip_amd.data_config, VERDICT r2 "missing" 1) on raw
`.npy` clips and frame directories, host side only (no GPU here):

* ViViT / TimeSformer: `create_dataloaders(args, sampling_methods, logger)` -> (loaders, class labels);
  batches are the reference `video_collate_fn` dicts, the clips hold the frames at the indices the
  pinned sampler draws in call order (vivit dataset.py:129-193; the sampler itself is pinned to the
  reference's goldens in tests/test_sampling_golden.py), with 0 and 2 worker processes.
* Swin3D / ResNet3D: the host half of `__getitem__` (`load_span`) decodes exactly the span
  `get_clip(idx[0] / fps, (idx[-1] + 1) / fps)` bounds, through the loaders' own worker DataLoader;
  ResNet3D's `sampled_frames_<mode>_<method>.csv` (dataset.py:245-289); `video_collate_fn` shapes.
"""
import argparse
import csv
import logging
import random

import numpy as np
import pytest
import torch

from vclip_amd import sampling
from vclip_amd.data_config import resnet3d, swin, timesformer, vivit

LOG = logging.getLogger("test_data_config")


def _clip(total, hw=(224, 224)):
    """uint8 [total, H, W, 3] whose frame i is filled with (i % 256, i // 256, 7): the frame number
    can be read back from any decoded pixel."""
    f = np.zeros((total, hw[0], hw[1], 3), np.uint8)
    f[..., 0] = (np.arange(total) % 256)[:, None, None]
    f[..., 1] = (np.arange(total) // 256)[:, None, None]
    f[..., 2] = 7
    return f


def _frame_ids(frames):
    return [int(fr[0, 0, 0]) + 256 * int(fr[0, 0, 1]) for fr in frames]


def _args(root, **kw):
    a = dict(data_dir=str(root), test_data_dir=None, num_frames=8, batch_size=2, num_workers=0,
             train_sampling="random_window", val_sampling="uniform", test_sampling="random")
    a.update(kw)
    return argparse.Namespace(**a)


@pytest.fixture(scope="module")
def npy_root(tmp_path_factory):
    """<root>/{train,val,test}/{non-referral,referral}/*.npy, 224x224 clips of 5-40 frames."""
    root = tmp_path_factory.mktemp("npy")
    totals = {"train": [40, 5, 33, 12], "val": [9, 20], "test": [31, 8]}
    for split, ts in totals.items():
        for k, t in enumerate(ts):
            d = root / split / ("referral" if k % 2 else "non-referral")
            d.mkdir(parents=True, exist_ok=True)
            np.save(d / f"{split}{k}.npy", _clip(t))
    return root


@pytest.mark.parametrize("folder", [vivit, timesformer])
def test_hf_folder_loaders_follow_the_sampler_in_call_order(npy_root, folder):
    loaders, labels = folder.create_dataloaders(_args(npy_root), {"train": "random_window", "val": "uniform",
                                                                  "test": "random"}, LOG)
    assert labels == ["non-referral", "referral"]
    # test split (no shuffle): the global stream seeded 42 by the LAST dataset constructed (test)
    ds = loaders["test"].dataset
    random.seed(42)
    np.random.seed(42)
    expect = [sampling.sample_indices(np.load(p, mmap_mode="r").shape[0], 8, "random") for p in ds.video_paths]
    random.seed(42)
    np.random.seed(42)
    got = []
    for b in loaders["test"]:
        pv = b["pixel_values"]
        pv = list(pv) if isinstance(pv, list) else list(pv.numpy())  # ViViT's test loader: default collate
        assert all(c.shape == (8, 224, 224, 3) and c.dtype == np.uint8 for c in pv)
        got += [_frame_ids(c) for c in pv]
        assert b["labels"].dtype == torch.long
    assert got == expect
    assert len(loaders["train"]) == 2 and len(loaders["val"]) == 1


def test_vivit_loader_workers_match_serial(npy_root):
    """--num_workers takes effect: 2 decode workers give the same (uniform, deterministic) batches."""
    outs = []
    for nw in (0, 2):
        loaders, _ = vivit.create_dataloaders(_args(npy_root, num_workers=nw), {"train": "uniform", "val": "uniform",
                                                                                  "test": "uniform"}, LOG)
        assert loaders["val"].num_workers == nw
        outs.append([np.stack(b["pixel_values"]) for b in loaders["val"]])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_timesformer_inference_mode(npy_root):
    p = sorted((npy_root / "test" / "non-referral").iterdir())[0]
    ds = timesformer.VideoDataset(str(p), mode="inference", num_frames=8)
    assert len(ds) == 1 and ds.labels == [0]
    item = ds[0]
    assert item["pixel_values"].shape == (8, 224, 224, 3) and _frame_ids(item["pixel_values"]) == \
        sampling.sample_indices(31, 8, "uniform")


def _span_case(root, names_totals, fps=None):
    d = root / "val" / "referral"
    d.mkdir(parents=True)
    for name, total in names_totals:
        np.save(d / name, _clip(total, (8, 8)))
        if fps:
            (d / name).with_suffix(".fps").write_text(str(fps))


@pytest.mark.parametrize("fps", [30.0, 25.0])
def test_swin_span_is_the_sampled_window(tmp_path, fps):
    """Swin3D divides by the video's own fps: the span is exactly frames idx[0] .. idx[-1]."""
    _span_case(tmp_path, [("a.npy", 40), ("b.npy", 5), ("c.npy", 100)], fps=fps)
    ds = swin.VideoDataset(str(tmp_path), mode="val", sampling_method="random_window", num_frames=8, logger=LOG)
    seen = []
    orig = ds._sampler.get_sampling_indices
    ds._sampler.get_sampling_indices = lambda p, t: seen.append(orig(p, t)) or seen[-1]
    random.seed(42)
    expect = [sampling.sample_indices(np.load(p, mmap_mode="r").shape[0], 8, "random_window") for p in ds.video_paths]
    random.seed(42)
    loader = swin.DeviceClipLoader(ds, batch_size=2)
    spans = [fr for batch in loader.loader for fr, label in batch]
    assert [s[0] for s in seen] == expect
    for span, idx in zip(spans, expect):
        assert _frame_ids(span) == list(range(idx[0], idx[-1] + 1))
    assert len(loader) == 2


def test_resnet3d_span_uses_constant_30fps_and_writes_csv(tmp_path):
    """ResNet3D divides by its constant fps = 30 whatever the video's rate (dataset.py:219-222): at a
    real 60 fps the decoded span covers twice the sampled frame numbers.  The CSV holds the cached
    indices (hash(basename) seeding, vclip_amd.sampling.Resnet3dSampler) in sorted path order."""
    _span_case(tmp_path, [("v00007.npy", 64), ("v00020.npy", 20)], fps=60.0)
    log_dir = tmp_path / "logs"
    log_dir.mkdir()
    ds = resnet3d.VideoDataset(str(tmp_path), mode="val", sampling_method="random", num_frames=8, logger=LOG,
                               log_dir=str(log_dir))
    ref = sampling.Resnet3dSampler(8, "random", seed=False)
    expect = {p: ref.get_sampling_indices(p, np.load(p, mmap_mode="r").shape[0]) for p in ds.video_paths}
    path = ds.save_sampled_indices()
    rows = list(csv.reader(open(path)))
    assert path.endswith("sampled_frames_val_random.csv") and rows[0] == ["video_filename", "total_frames",
                                                                          "sampled_frames"]
    for row, p in zip(rows[1:], sorted(ds.video_paths)):
        assert row[0] == p.split("/")[-1] and row[2] == ",".join(map(str, expect[p]))
    for i, p in enumerate(ds.video_paths):
        span, label = ds.load_span(i)
        idx, total = expect[p], np.load(p, mmap_mode="r").shape[0]
        lo, hi = int(np.ceil(idx[0] / 30 * 60 - 1e-6)), min(total, int(np.ceil((idx[-1] + 1) / 30 * 60 - 1e-6)))
        assert _frame_ids(span) == list(range(lo, hi)) and label == 1


def test_span_dataset_refuses_gpu_transform_in_a_worker(tmp_path):
    _span_case(tmp_path, [("a.npy", 12)])
    ds = swin.VideoDataset(str(tmp_path), mode="val", num_frames=8, logger=LOG)
    loader = torch.utils.data.DataLoader(ds, batch_size=1, num_workers=1)
    with pytest.raises(RuntimeError, match="DataLoader worker"):
        next(iter(loader))


def test_span_collate_shapes():
    batch = [(torch.zeros(1, 3, 8, 224, 224), torch.tensor([1])), (torch.ones(2, 3, 8, 224, 224), torch.tensor([0, 0]))]
    clips, labels = swin.video_collate_fn(batch)
    assert clips.shape == (2, 1, 3, 8, 224, 224) and labels.shape == (2, 1)
    assert resnet3d.video_collate_fn is swin.video_collate_fn
