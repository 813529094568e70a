"""Oracle self-checks for the byte/layout restatements (CPU)."""
import numpy as np
import torch

from oracle.frames_ref import gather_norm, gather_u8, tubelet_im2col
from vclip_amd.weights import frames_to_pixel_values, make_synthetic_frames


def test_gather_matches_dataset_semantics():
    fr = make_synthetic_frames(2, 40, 16, seed=3)
    idx = np.array([[0, 5, 39, 60, -2], [1, 1, 2, 3, 39]])
    g = gather_u8(fr, idx)
    assert g.shape == (2, 5, 16, 16, 3)
    assert (g[0, 3] == fr[0, 39]).all() and (g[0, 4] == fr[0, 0]).all()  # clamped both ways


def test_gather_norm_is_processor_affine():
    fr = make_synthetic_frames(1, 8, 16, seed=4)
    idx = np.arange(8)[None]
    np.testing.assert_array_equal(gather_norm(fr, idx), frames_to_pixel_values(fr))
    v = gather_norm(fr, idx)
    assert v.min() >= -3.0 and v.max() <= 1.0


def test_im2col_is_conv3d():
    rng = np.random.RandomState(0)
    pix = rng.standard_normal((2, 4, 3, 32, 32)).astype(np.float32)
    w = rng.standard_normal((5, 3, 2, 16, 16)).astype(np.float32)
    A = tubelet_im2col(pix)
    ref = torch.nn.functional.conv3d(torch.from_numpy(pix).transpose(1, 2), torch.from_numpy(w), stride=(2, 16, 16))
    ref = ref.flatten(2).transpose(1, 2).reshape(-1, 5).numpy()
    np.testing.assert_allclose(A @ w.reshape(5, -1).T, ref, atol=1e-3)
