"""`vivit_transformer/vivit_classifier/data_config/` drop-in: `VideoDataset` (dataset.py:10-381, the
class in vclip_amd/video_dataset.py), `video_collate_fn` (dataloader.py:6-50) and
`create_dataloaders(args, sampling_methods, logger)` (dataloader.py:52-135)."""
from __future__ import annotations

import numpy as np
import torch
from torch.utils.data import DataLoader

from ..video_dataset import VideoDataset

__all__ = ["VideoDataset", "video_collate_fn", "create_dataloaders"]


def video_collate_fn(batch, num_frames=32):
    """{'pixel_values': list of uint8 [T, H, W, 3] numpy clips, 'labels': stacked labels}.  A clip that
    is not [T, H, W, 3] is squeezed, and replaced by a zero [32, 224, 224, 3] placeholder with a
    printed warning when that does not fix it (dataloader.py:6-50)."""
    pixel_values, labels = [], []
    for sample in batch:
        if sample.get("pixel_values") is not None:
            frames = sample["pixel_values"]
            if isinstance(frames, torch.Tensor):
                frames = frames.cpu().numpy()
            if frames.ndim == 4 and frames.shape[-1] == 3:
                pixel_values.append(frames)
            else:
                fixed = np.squeeze(frames)
                if fixed.ndim == 4 and fixed.shape[-1] == 3:
                    pixel_values.append(fixed)
                else:
                    print(f"Warning: Could not fix frame shape {frames.shape}, using placeholder")
                    pixel_values.append(np.zeros((num_frames, 224, 224, 3), dtype=np.uint8))
        if sample.get("labels") is not None:
            labels.append(sample["labels"])
    labels = torch.stack(labels) if labels else torch.zeros(len(batch), dtype=torch.long)
    return {"pixel_values": pixel_values, "labels": labels}


def _create(dataset_cls, args, sampling_methods, logger, test_collate):
    logger.info(f"Creating datasets from {args.data_dir}")
    logger.info(f"Using sampling methods: {sampling_methods}")
    datasets, dataloaders, class_labels = {}, {}, None
    for split in ("train", "val"):
        try:
            datasets[split] = dataset_cls(args.data_dir, mode=split, sampling_method=sampling_methods[split],
                                          num_frames=args.num_frames, logger=logger)
            if class_labels is None:
                class_labels = datasets[split].class_labels
                logger.info(f"Detected class labels: {class_labels}")
            dataloaders[split] = DataLoader(datasets[split], batch_size=args.batch_size, shuffle=(split == "train"),
                                            num_workers=args.num_workers, pin_memory=torch.cuda.is_available(),
                                            collate_fn=video_collate_fn)
            logger.info(f"Created {split} dataloader with {len(dataloaders[split])} batches (batch size: "
                        f"{args.batch_size}) using {sampling_methods[split]} sampling")
        except Exception as e:
            logger.error(f"Error creating {split} dataset/dataloader: {str(e)}")
            raise
    try:
        test_data_dir = args.test_data_dir if args.test_data_dir else args.data_dir
        datasets["test"] = dataset_cls(test_data_dir, mode="test", sampling_method=sampling_methods["test"],
                                       num_frames=args.num_frames, logger=logger)
        # ViViT's test loader has no collate_fn (dataloader.py:116-123): torch's default collate
        kw = {"collate_fn": video_collate_fn} if test_collate else {}
        dataloaders["test"] = DataLoader(datasets["test"], batch_size=args.batch_size, shuffle=False,
                                         num_workers=args.num_workers, pin_memory=torch.cuda.is_available(), **kw)
        logger.info(f"Created test dataloader from {test_data_dir} with {len(dataloaders['test'])} batches (batch "
                    f"size: {args.batch_size}) using {sampling_methods['test']} sampling")
    except Exception as e:
        logger.error(f"Error creating test dataset/dataloader: {str(e)}")
        raise
    return dataloaders, class_labels


def create_dataloaders(args, sampling_methods, logger):
    """(dataloaders {'train', 'val', 'test'}, class_labels); args: data_dir, test_data_dir,
    num_frames, batch_size, num_workers (dataloader.py:52-135)."""
    return _create(VideoDataset, args, sampling_methods, logger, test_collate=False)
