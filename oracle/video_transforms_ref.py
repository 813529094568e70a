"""CPU oracle (test infrastructure only) of the Swin3D / ResNet3D train-time clip transforms,
videoswintransformer/swin_video_classifier/data_config/dataset.py:151-163 (train branch):

    UniformTemporalSubsample(T) -> RandomShortSideScale(256, 320) -> RandomCrop(224)
    -> RandomHorizontalFlip(0.5) -> Normalize((0.45,)*3, (0.225,)*3)

applied to the float [C, T, H, W] clip of one __getitem__ call.  pytorchvideo (0.1.5) and
torchvision are absent from this image, so their published algorithms are restated here --
parity unpinned:
  * pytorchvideo.transforms.functional.uniform_temporal_subsample: torch.linspace(0, t - 1, T)
    .clamp(0, t - 1).long() along the time axis;
  * RandomShortSideScale.__call__: size = torch.randint(min_size, max_size + 1, (1,)).item(), then
    short_side_scale(x, size, "bilinear"): the short side becomes `size`, the long side
    int(math.floor(long / short * size)), torch.nn.functional.interpolate(mode="bilinear",
    align_corners=False) over (H, W);
  * torchvision RandomCrop.get_params: i = torch.randint(0, h - th + 1, size=(1,)).item(), then
    j likewise over w (returns (0, 0) without drawing when the frame already is th x tw);
  * RandomHorizontalFlip.forward: torch.rand(1) < p -> flip the last axis;
  * Normalize: (x - mean[c]) / std[c] per channel (the datasets pass 0-255 values: no /255).
"""
import math

import torch


def uniform_temporal_subsample(x, num_samples):
    t = x.shape[1]
    idx = torch.linspace(0, t - 1, num_samples).clamp(0, t - 1).long()
    return x[:, idx]


def short_side_scale(x, size):
    c, t, h, w = x.shape
    if w < h:
        new_h, new_w = int(math.floor((float(h) / w) * size)), size
    else:
        new_h, new_w = size, int(math.floor((float(w) / h) * size))
    return torch.nn.functional.interpolate(x, size=(new_h, new_w), mode="bilinear", align_corners=False)


def train_transform(clip_u8_thwc, num_frames, min_size=256, max_size=320, crop=224, p_flip=0.5,
                    mean=(0.45, 0.45, 0.45), std=(0.225, 0.225, 0.225), generator=None):
    """One clip: uint8 [F, H, W, 3] -> (f32 [3, T, crop, crop], (resize_h, resize_w, top, left, flip))."""
    x = clip_u8_thwc.permute(3, 0, 1, 2).float()  # [C, F, H, W]
    x = uniform_temporal_subsample(x, num_frames)
    size = torch.randint(min_size, max_size + 1, (1,), generator=generator).item()
    x = short_side_scale(x, size)
    h, w = x.shape[-2:]
    if h == crop and w == crop:
        i = j = 0
    else:
        i = torch.randint(0, h - crop + 1, size=(1,), generator=generator).item()
        j = torch.randint(0, w - crop + 1, size=(1,), generator=generator).item()
    x = x[..., i:i + crop, j:j + crop]
    flip = bool(torch.rand(1, generator=generator) < p_flip)
    if flip:
        x = x.flip(-1)
    m = torch.tensor(mean).view(3, 1, 1, 1)
    s = torch.tensor(std).view(3, 1, 1, 1)
    return (x - m) / s, (h, w, i, j, int(flip))
