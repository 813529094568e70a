"""GPU preprocessing vs the reference's own transforms: Pillow (bit-exact uint8 resize),
transformers VivitImageProcessor (the ViViT trainer's processor), and the pytorchvideo
eval chain restated with torch ops (F.interpolate bilinear, CenterCrop, Normalize)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
PIL = pytest.importorskip("PIL.Image")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vclip_amd import _lib
    _lib.load()


@pytest.mark.parametrize("H,W,H2,W2", [(224, 224, 256, 256), (240, 320, 256, 341), (300, 200, 200, 133)])
def test_pil_resize_bit_exact(H, W, H2, W2):
    from vclip_amd.preprocess import pil_resize_u8
    rng = np.random.RandomState(H * W)
    imgs = rng.randint(0, 256, (3, H, W, 3)).astype(np.uint8)
    got = pil_resize_u8(torch.from_numpy(imgs).to(DEV), (H2, W2)).cpu().numpy()
    for i in range(3):
        ref = np.asarray(PIL.fromarray(imgs[i]).resize((W2, H2), PIL.BILINEAR))
        assert np.array_equal(got[i], ref)


def test_vivit_preprocess_vs_hf_processor():
    transformers = pytest.importorskip("transformers")
    from vclip_amd.preprocess import vivit_preprocess
    proc = transformers.VivitImageProcessor(num_frames=4, image_size=224, patch_size=16)
    rng = np.random.RandomState(1)
    frames = rng.randint(0, 256, (2, 4, 224, 224, 3)).astype(np.uint8)
    want = np.concatenate([proc(list(frames[b]), return_tensors="np")["pixel_values"] for b in range(2)])
    got = vivit_preprocess(torch.from_numpy(frames).to(DEV)).cpu().numpy()
    assert got.shape == want.shape
    assert np.abs(got - want).max() < 1e-5


def test_timesformer_preprocess_vs_hf_processor():
    """timesformer trainer.py:91-97: the facebook/timesformer-base-finetuned-k400 processor
    (VideoMAEImageProcessor: mean / std 0.45 / 0.225, resize + centre crop to 224 x 224, x / 255)
    on 224 x 224 frames, per clip; built locally with that checkpoint's settings (no hub)."""
    transformers = pytest.importorskip("transformers")
    from vclip_amd.preprocess import timesformer_preprocess
    cls = getattr(transformers, "VideoMAEImageProcessorPil", None) or transformers.VideoMAEImageProcessor
    proc = cls(size={"height": 224, "width": 224}, crop_size={"height": 224, "width": 224},
               image_mean=[0.45, 0.45, 0.45], image_std=[0.225, 0.225, 0.225])
    rng = np.random.RandomState(2)
    frames = rng.randint(0, 256, (2, 8, 224, 224, 3)).astype(np.uint8)
    want = np.concatenate([proc(images=list(frames[b]), return_tensors="np", do_resize=True,
                                size={"height": 224, "width": 224}, do_center_crop=True,
                                crop_size={"height": 224, "width": 224})["pixel_values"] for b in range(2)])
    got = timesformer_preprocess(torch.from_numpy(frames).to(DEV)).cpu().numpy()
    assert got.shape == want.shape
    assert np.abs(got - want).max() < 1e-5


@pytest.mark.parametrize("F,H,W,T,div255", [(40, 240, 320, 16, False), (12, 224, 224, 32, True), (9, 300, 256, 8, False)])
def test_video_eval_transform(F, H, W, T, div255):
    from vclip_amd.preprocess import short_side_size, uniform_temporal_subsample_indices, video_eval_transform
    rng = np.random.RandomState(F)
    frames = rng.randint(0, 256, (2, F, H, W, 3)).astype(np.uint8)
    got = video_eval_transform(torch.from_numpy(frames).to(DEV), T, div255=div255).cpu()
    x = torch.from_numpy(frames).float().permute(0, 4, 1, 2, 3)  # [B, C, F, H, W] as EncodedVideo gives
    x = x[:, :, uniform_temporal_subsample_indices(F, T)]
    rh, rw = short_side_size(H, W, 256)
    B = x.shape[0]
    x = torch.nn.functional.interpolate(x.reshape(B * 3, T, H, W), size=(rh, rw), mode="bilinear",
                                        align_corners=False).reshape(B, 3, T, rh, rw)
    top, left = int(round((rh - 224) / 2.0)), int(round((rw - 224) / 2.0))
    x = x[..., top:top + 224, left:left + 224]
    if div255:
        x = x / 255.0
    want = (x - 0.45) / 0.225
    tol = 1e-4 * (1.0 if div255 else 255.0)
    assert got.shape == want.shape and (got - want).abs().max().item() < tol


@pytest.mark.parametrize("shape", [(48, 64, 224, 224), (240, 320, 224, 224), (448, 448, 224, 224), (100, 90, 224, 224),
                                   (17, 23, 11, 7), (7, 5, 10, 13)])
def test_cv2_resize_gpu_bit_exact(shape):
    """vc_resize_linear_u8 == the host restatement of cv2.resize INTER_LINEAR (vclip_amd/resize.py), which
    tests/test_video_dataset.py pins to the loop oracle (oracle/cv2_resize_ref.py); parity with cv2 itself
    is unpinned (cv2 absent from the image).  448 -> 224 is the exact-2x INTER_AREA path."""
    from vclip_amd import preprocess
    from vclip_amd.resize import resize_linear_u8
    H, W, h, w = shape
    x = np.random.RandomState(H + W).randint(0, 256, (3, H, W, 3)).astype(np.uint8)
    got = preprocess.cv2_resize_u8(torch.from_numpy(x).cuda(), (w, h)).cpu().numpy()
    np.testing.assert_array_equal(got, resize_linear_u8(x, (w, h)))
    if H * W * h * w < 2e6:
        from oracle.cv2_resize_ref import resize_linear_u8 as ref
        np.testing.assert_array_equal(got[0], np.array(ref(x[0].tolist(), w, h), dtype=np.uint8))


@pytest.mark.parametrize("F,H,W,T", [(40, 240, 320, 16), (12, 224, 224, 8), (9, 300, 256, 8)])
def test_video_train_transform(F, H, W, T):
    """RandomShortSideScale -> RandomCrop -> RandomHorizontalFlip -> Normalize on the GPU (parameters
    drawn on the host) vs the CPU restatement of the pytorchvideo / torchvision chain with the same
    generator seed (oracle/video_transforms_ref.py; parity unpinned: neither library is installed)."""
    from oracle.video_transforms_ref import train_transform
    from vclip_amd.preprocess import video_train_transform
    rng = np.random.RandomState(F + H)
    frames = rng.randint(0, 256, (3, F, H, W, 3)).astype(np.uint8)
    got, params = video_train_transform(torch.from_numpy(frames).to(DEV), T, generator=torch.Generator().manual_seed(7))
    g = torch.Generator().manual_seed(7)
    for b in range(3):
        want, p = train_transform(torch.from_numpy(frames[b]), T, generator=g)
        assert list(p) == params[b].tolist()
        assert (got[b].cpu() - want).abs().max().item() < 1e-4 * 255.0
