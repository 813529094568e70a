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
