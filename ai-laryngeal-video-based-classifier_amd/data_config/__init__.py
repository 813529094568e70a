"""Per-folder dataset / DataLoader drop-ins: the reference's `<pkg>/data_config/{dataset,dataloader}.py`
of each of the four model folders, same class / function names, constructor arguments, item and batch
formats:

  vclip_amd.data_config.vivit        vivit_transformer/vivit_classifier/data_config/
  vclip_amd.data_config.timesformer  timesformer/timesformer_classifier/data_config/
  vclip_amd.data_config.swin         videoswintransformer/swin_video_classifier/data_config/
  vclip_amd.data_config.resnet3d     resnet50-3d-video/video_classifier/data_config/

each exporting `VideoDataset`, `video_collate_fn` and `create_dataloaders` with the reference's signature.

Where the work runs: sampling (bit-exact, vclip_amd.sampling) and decode are host work in the
DataLoader's worker processes (`num_workers`), as in the reference.  The Swin3D / ResNet3D datasets
transform their clips inside `__getitem__` (UniformTemporalSubsample, short-side scale, crop, flip,
Normalize); here that transform is one fused GPU kernel (vc_video_transform_clips), which a forked
worker cannot launch, so their `create_dataloaders` returns a `DeviceClipLoader`: the workers do the
host half of `__getitem__` (`load_span`), the main process transforms each clip on the GPU and
collates exactly as the reference collate does.  Indexing such a dataset directly in the main process
(`ds[i]`) runs both halves and returns the reference item.  ViViT / TimeSformer items are the decoded
uint8 frames themselves (their processors run in the trainer, on the GPU in this build).
"""
from . import resnet3d, swin, timesformer, vivit
from ._device import DeviceClipLoader

FOLDERS = {"vivit": vivit, "timesformer": timesformer, "swin": swin, "resnet3d": resnet3d}

__all__ = ["FOLDERS", "DeviceClipLoader", "vivit", "timesformer", "swin", "resnet3d"]
