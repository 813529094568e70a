"""TimeSformer (divided space-time attention) on the GPU: kernels vs fp32 torch references,
and the end-to-end HIP path vs goldens made by HF transformers' TimesformerForVideoClassification
(tests/golden/timesformer_{tiny.npz,full.json}).  Logit tolerance 1e-2 (bf16, north_star)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle.frames_ref import tubelet_im2col
from vclip_amd.weights import make_synthetic_clips, make_timesformer_weights

pytestmark = pytest.mark.gpu
GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vclip_amd import _lib
    _lib.load()


def ops():
    from vclip_amd import ops as O
    return O


def test_patch_im2col_patch_major_bit_exact():
    rng = np.random.RandomState(3)
    B, T, H = 2, 8, 64
    pix = rng.standard_normal((B, T, 3, H, H)).astype(np.float32)
    n = B * T * (H // 16) ** 2
    out = torch.zeros((n + 32, 768), dtype=torch.bfloat16, device=DEV)
    ops().tubelet_im2col(torch.from_numpy(pix).to(DEV), (1, 16, 16), out, order="patch_major")
    ref = torch.from_numpy(tubelet_im2col(pix, (1, 16, 16), order="patch_major")).bfloat16()
    assert torch.equal(out[:n].cpu(), ref)


def _clip_rows(B, P, T):
    return B * (1 + P * T)


@pytest.mark.parametrize("B,P,T,H,pre", [(2, 16, 4, 2, False), (3, 196, 8, 12, True), (1, 5, 1, 1, False),
                                         (2, 7, 16, 2, True), (2, 5, 16, 8, False), (2, 5, 12, 10, True),
                                         (1, 3, 16, 12, True), (2, 3, 32, 2, False)])
def test_temporal_attention(B, P, T, H, pre):
    """LDS kernel (one workgroup per patch) when T <= 16 and the patch's q|k|v rows fit 64 KB
    (T*H <= 128 pairs in one pass, more in a loop); thread-per-query kernel otherwise
    ((1, 3, 16, 12): 72 KB; T = 32)."""
    g = torch.Generator().manual_seed(B * 1000 + P + T)
    S = 1 + P * T
    rows = B * S + 8
    qkv = (torch.randn(rows, 3 * H * 64, generator=g) * 1.5).bfloat16()
    scale = 0.125
    if pre:
        qkv[:, :H * 64] = (qkv[:, :H * 64].float() * scale * 1.4426950408889634).bfloat16()
    out = torch.zeros(rows, H * 64, dtype=torch.bfloat16, device=DEV)
    ops().temporal_attention(qkv.to(DEV), B, P, T, H, scale, out, q_prescaled=pre)
    q = qkv.float()
    x = torch.stack([q[b * S + 1: (b + 1) * S] for b in range(B)]).view(B * P, T, 3, H, 64)
    qq, kk, vv = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = qq @ kk.transpose(-1, -2)
    s = s / 1.4426950408889634 if pre else s * scale
    ref = (torch.softmax(s, -1) @ vv).transpose(1, 2).reshape(B, P * T, H * 64)
    o = out.float().cpu()
    got = torch.stack([o[b * S + 1: (b + 1) * S] for b in range(B)])
    assert (got - ref).abs().max().item() < 2e-2
    assert all(o[b * S].abs().sum().item() == 0 for b in range(B))  # CLS rows untouched


@pytest.mark.parametrize("D", [768, 128])
def test_divided_add_layernorm_modes(D):
    B, P, T = 2, 9, 4
    S = 1 + P * T
    g = torch.Generator().manual_seed(D)
    x0 = torch.randn(B * S + 3, D, generator=g)
    gam, bet = 1 + 0.1 * torch.randn(D, generator=g), 0.1 * torch.randn(D, generator=g)
    eps = 1e-6
    ln = lambda t: torch.nn.functional.layer_norm(t, (D,), gam, bet, eps)  # noqa: E731
    # mode 0: y in clip layout, h in frame layout
    y = torch.randn(B * S + 3, D, generator=g).bfloat16()
    x = x0.clone().to(DEV)
    h = torch.zeros(B * T * (1 + P) + 3, D, dtype=torch.bfloat16, device=DEV)
    ops().divided_add_layernorm(x, y.to(DEV), B, P, T, gam.to(DEV), bet.to(DEV), eps, "temporal_to_spatial", h)
    xr = x0.clone()
    for b in range(B):
        xr[b * S + 1:(b + 1) * S] += y[b * S + 1:(b + 1) * S].float()
    assert torch.allclose(x.cpu(), xr, atol=1e-6)
    hr = torch.zeros(B * T * (1 + P), D)
    for b in range(B):
        for t in range(T):
            hr[(b * T + t) * (1 + P)] = ln(xr[b * S])
            for p in range(P):
                hr[(b * T + t) * (1 + P) + 1 + p] = ln(xr[b * S + 1 + p * T + t])
    assert (h[:B * T * (1 + P)].float().cpu() - hr).abs().max().item() < 3e-2
    # mode 1: y in frame layout, h in clip layout, CLS gets the frame mean
    yf = torch.randn(B * T * (1 + P) + 3, D, generator=g).bfloat16()
    x = x0.clone().to(DEV)
    hc = torch.zeros(B * S + 3, D, dtype=torch.bfloat16, device=DEV)
    ops().divided_add_layernorm(x, yf.to(DEV), B, P, T, gam.to(DEV), bet.to(DEV), eps, "spatial_to_mlp", hc)
    xr = x0.clone()
    for b in range(B):
        xr[b * S] += torch.stack([yf[(b * T + t) * (1 + P)].float() for t in range(T)]).mean(0)
        for p in range(P):
            for t in range(T):
                xr[b * S + 1 + p * T + t] += yf[(b * T + t) * (1 + P) + 1 + p].float()
    assert torch.allclose(x.cpu(), xr, atol=1e-5)
    assert (hc[:B * S].float().cpu() - ln(xr[:B * S])).abs().max().item() < 3e-2


def _model(cfg):
    from vclip_amd.timesformer import TimesformerConfig, TimesformerForVideoClassification
    c = TimesformerConfig(**cfg, id2label={0: "non-referral", 1: "referral"})
    m = TimesformerForVideoClassification(c)
    m.load_state_dict(make_timesformer_weights(cfg, seed=0))
    return m.cuda().eval()  # constructed models start in train mode, as HF's (forward would then train)


def test_timesformer_tiny_logits():
    g = np.load(os.path.join(GD, "timesformer_tiny.npz"))
    cfg = json.loads(str(g["config"]))
    m = _model(cfg)
    lg = m(pixel_values=torch.from_numpy(g["pixel_values"]).cuda()).logits.cpu().numpy()
    err = np.abs(lg - g["logits"]).max()
    assert err < 1e-2, (err, lg, g["logits"])


def test_timesformer_b_full_logits():
    with open(os.path.join(GD, "timesformer_full.json")) as f:
        g = json.load(f)
    cfg = g["config"]
    m = _model(cfg)
    pix = make_synthetic_clips(g["batch"], cfg["num_frames"], cfg["image_size"], seed=g["input_seed"])
    lg = m(pixel_values=torch.from_numpy(pix).cuda()).logits.cpu().numpy()
    err = np.abs(lg - np.array(g["logits"])).max()
    assert err < 1e-2, (err, lg, g["logits"])


def test_timesformer_b_batch16_logits_configs2():
    """BASELINE configs[2] at its own workload: TimeSformer-B 8x224^2, batch 16, against transformers'
    TimesformerForVideoClassification at batch 16 (tests/golden/timesformer_b16.json), bf16 bar 1e-2."""
    with open(os.path.join(GD, "timesformer_b16.json")) as f:
        g = json.load(f)
    cfg = g["config"]
    m = _model(cfg)
    pix = torch.from_numpy(make_synthetic_clips(g["batch"], cfg["num_frames"], cfg["image_size"],
                                                seed=g["input_seed"])).cuda()
    lg = m(pixel_values=pix).logits.cpu().numpy()
    lf = m.forward_logits(pix).cpu().numpy()  # bench.py --mode timesformer's call
    ref = np.array(g["logits"])
    errs = (float(np.abs(lg - ref).max()), float(np.abs(lf - ref).max()))
    print("TimeSformer-B B=16 max |logit - HF golden| (model(), forward_logits):", errs)
    assert max(errs) < 1e-2, (errs, lg, ref)


def test_timesformer_batch_invariance():
    with open(os.path.join(GD, "timesformer_full.json")) as f:
        cfg = json.load(f)["config"]
    m = _model(cfg)
    pix = torch.from_numpy(make_synthetic_clips(3, cfg["num_frames"], cfg["image_size"], seed=5)).cuda()
    full = m(pixel_values=pix).logits.clone()
    one = m(pixel_values=pix[1:2].contiguous()).logits.clone()
    assert torch.equal(full[1:2], one)


def test_timesformer_two_stream_split_bit_exact():
    """concurrent_streams = 2 splits the batch over two HIP streams (vclip_amd.streams): logits
    equal the one-stream run bit for bit."""
    from vclip_amd.timesformer import create_model
    m = create_model(num_frames=8, device="cuda")
    pix = torch.from_numpy(make_synthetic_clips(5, 8, 224, seed=3)).cuda()
    m.concurrent_streams = 1
    one = m.forward_logits(pix).clone()
    m.concurrent_streams = 2
    two = m.forward_logits(pix).clone()
    assert torch.equal(one, two)
    # uneven parts (model.split_sizes) and a per-GEMM tile override (model.gemm_cfg): the same bits
    m.split_sizes = [4, 1]
    assert torch.equal(m.forward_logits(pix), one)
    m.concurrent_streams, m.split_sizes = 1, None
    m.gemm_cfg = {"fc1": 8, "fc2": 8}
    assert torch.equal(m.forward_logits(pix), one)


@pytest.mark.parametrize("streams", [1, 2])
def test_timesformer_graph_replay_bit_identical(streams):
    """forward_logits replayed from its captured hipGraph (model.graph_replay) == the eager forward,
    bit for bit, including after an in-place update of the captured input."""
    g = np.load(os.path.join(GD, "timesformer_tiny.npz"))
    m = _model(json.loads(str(g["config"])))
    m.concurrent_streams = streams
    pix = torch.from_numpy(g["pixel_values"]).cuda()
    pix2 = torch.flip(pix, dims=[0]).contiguous()
    eager = [m.forward_logits(p).clone() for p in (pix, pix2)]
    m.graph_replay = True
    buf = pix.clone()
    for _ in range(2):
        assert torch.equal(m.forward_logits(buf), eager[0])
    buf.copy_(pix2)
    assert torch.equal(m.forward_logits(buf), eager[1])
