"""Host side of the preprocessing path: Pillow's fixed-point coefficient tables (what the GPU
resampler consumes) restated and checked bit-exact against Pillow itself; pytorchvideo's
UniformTemporalSubsample indices; resize geometry."""
import numpy as np
import pytest
import torch

from oracle.frames_ref import pil_resize_emulated
from vclip_amd.preprocess import pil_bilinear_coeffs, short_side_size, uniform_temporal_subsample_indices

PIL = pytest.importorskip("PIL.Image")


@pytest.mark.parametrize("H,W,H2,W2", [(224, 224, 256, 256), (240, 320, 256, 341), (300, 200, 200, 133),
                                       (64, 48, 64, 97)])
def test_pil_coeffs_bit_exact_vs_pillow(H, W, H2, W2):
    rng = np.random.RandomState(H + W)
    img = rng.randint(0, 256, (H, W, 3)).astype(np.uint8)
    ref = np.asarray(PIL.fromarray(img).resize((W2, H2), PIL.BILINEAR))
    assert np.array_equal(pil_resize_emulated(img, (H2, W2), pil_bilinear_coeffs), ref)


def test_uniform_temporal_subsample():
    for t, T in [(300, 32), (20, 32), (8, 8), (1, 4), (97, 16)]:
        idx = uniform_temporal_subsample_indices(t, T)
        want = torch.linspace(0, t - 1, T).clamp(0, t - 1).long()
        assert torch.equal(idx, want) and idx.min() >= 0 and idx.max() <= t - 1


def test_short_side_size():
    assert short_side_size(480, 640, 256) == (256, 341)
    assert short_side_size(640, 480, 256) == (341, 256)
    assert short_side_size(224, 224, 256) == (256, 256)


@pytest.mark.parametrize("H,W", [(240, 320), (320, 240), (256, 256), (224, 224)])
def test_train_transform_params_draw_order(H, W):
    """The host draw of the train chain's parameters consumes torch's RNG exactly as the
    restated pytorchvideo / torchvision transforms do (oracle/video_transforms_ref.py), clip
    after clip, and yields the same sizes, crop windows and flips."""
    from oracle.video_transforms_ref import train_transform
    from vclip_amd.preprocess import train_transform_params
    clip = torch.zeros(4, H, W, 3, dtype=torch.uint8)
    g1, g2 = torch.Generator().manual_seed(123), torch.Generator().manual_seed(123)
    got = train_transform_params(6, H, W, generator=g1).tolist()
    want = [list(train_transform(clip, 2, generator=g2)[1]) for _ in range(6)]
    assert got == want
    assert torch.rand(1, generator=g1).item() == torch.rand(1, generator=g2).item()  # same RNG position after
    assert all(r[0] >= 224 and r[1] >= 224 for r in got)
