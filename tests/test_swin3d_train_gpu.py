"""Swin3D train step (videoswintransformer/swin_video_classifier/trainers/trainer.py:105-122:
model.train(), outputs = model(videos), CrossEntropyLoss, loss.backward(), AdamW.step()) on the
HIP autograd ops, against fp32 torch autograd of oracle/swin3d_ref.py (the restatement of
torchvision's swin3d; torchvision is absent, so parity with the library itself is UNPINNED).

Tolerances as the ViViT / TimeSformer train tests: bf16 operands with fp32 accumulation, so
per-parameter gradients by relative L2 (<= 5e-2) and cosine (>= 0.998); logits 1e-2 absolute.
Stochastic depth (random by design) is switched off for the gradient comparisons."""
import numpy as np
import pytest
import torch

from oracle import swin3d_ref as ref
from vclip_amd.weights import make_swin3d_weights, make_synthetic_video

pytestmark = pytest.mark.gpu
DEV = "cuda"

TINY = dict(patch_size=(2, 4, 4), embed_dim=32, depths=(2, 2), num_heads=(1, 2), window_size=(2, 3, 3),
            mlp_ratio=4.0, layer_norm_eps=1e-5, num_classes=2)
# Swin-T stage-1 geometry: 96 channels, 3 heads, the (8, 7, 7) window with its (4, 3, 3) shift
STAGE1 = dict(TINY, embed_dim=96, depths=(2,), num_heads=(3,), window_size=(8, 7, 7))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vclip_amd import _lib
    _lib.load()


def _attn_ref(qkv, table, B, grid, heads, window, shift, full):
    """fp32 torch of what the kernel computes: q' prescaled (d^-1/2 log2 e) q|k|v rows in token
    order, torchvision's roll / partition / bias / shift mask / softmax / reverse (oracle helpers)."""
    T, H, W = grid
    C = heads * 32
    x = qkv.reshape(B, T, H, W, 3 * C)
    if sum(shift):
        x = torch.roll(x, shifts=(-shift[0], -shift[1], -shift[2]), dims=(1, 2, 3))
    wt, wh, ww = window
    nw = (T // wt) * (H // wh) * (W // ww)
    vol = wt * wh * ww
    x = x.view(B, T // wt, wt, H // wh, wh, W // ww, ww, 3 * C).permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(B * nw, vol, 3 * C)
    q, k, v = x.reshape(B * nw, vol, 3, heads, 32).permute(2, 0, 3, 1, 4)
    attn = (q @ k.transpose(-2, -1)) / ref_log2e() + ref.relative_position_bias(table, full, window).unsqueeze(0)
    if sum(shift):
        m = ref.shift_region_labels((T, H, W), window, shift)
        m = m.view(T // wt, wt, H // wh, wh, W // ww, ww).permute(0, 2, 4, 1, 3, 5).reshape(nw, vol)
        m = (m.unsqueeze(1) - m.unsqueeze(2)) != 0
        attn = attn.view(B, nw, heads, vol, vol).masked_fill(m.unsqueeze(1).unsqueeze(0), -100.0).view(-1, heads, vol, vol)
    o = torch.softmax(attn, -1) @ v
    o = o.transpose(1, 2).reshape(B, T // wt, H // wh, W // ww, wt, wh, ww, C)
    o = o.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(B, T, H, W, C)
    if sum(shift):
        o = torch.roll(o, shifts=tuple(shift), dims=(1, 2, 3))
    return o.reshape(B * T * H * W, C)


def ref_log2e():
    return 1.4426950408889634


@pytest.mark.parametrize("B,grid,heads,window,shift,full", [
    (2, (4, 6, 6), 1, (2, 3, 3), (0, 0, 0), (2, 3, 3)),
    (2, (4, 6, 6), 2, (2, 3, 3), (1, 1, 1), (2, 3, 3)),
    (1, (16, 14, 14), 3, (8, 7, 7), (4, 3, 3), (8, 7, 7)),   # Swin-T stage 1 window, shifted
    (1, (8, 7, 7), 2, (8, 7, 7), (4, 0, 0), (8, 7, 7)),      # window == grid in h, w (stage 4: shift dropped)
    (2, (4, 3, 3), 2, (2, 3, 3), (1, 0, 0), (2, 7, 7)),      # shrunk window: the full index sliced [:vol, :vol]
])
def test_window_attention_backward_vs_autograd(B, grid, heads, window, shift, full):
    from vclip_amd import autograd_ops as A
    T, H, W = grid
    rows = B * T * H * W
    ntab = (2 * full[0] - 1) * (2 * full[1] - 1) * (2 * full[2] - 1)
    g = torch.Generator().manual_seed(rows + heads)
    qkv = (torch.randn(rows, 3 * heads * 32, generator=g) * 0.7).bfloat16()
    table = torch.randn(ntab, heads, generator=g) * 0.5
    dout = torch.randn(rows, heads * 32, generator=g).bfloat16()
    xq = qkv.to(DEV).requires_grad_()
    tq = table.to(DEV).requires_grad_()
    o = A.window_attention(xq, tq, B, grid, heads, window, shift, full)
    o.backward(dout.to(DEV))
    xr = qkv.float().requires_grad_()
    tr = table.clone().requires_grad_()
    orf = _attn_ref(xr, tr, B, grid, heads, window, shift, full)
    orf.backward(dout.float())
    assert (o.float().cpu() - orf.detach()).abs().max().item() < 2e-2
    for got, want, nm in ((xq.grad.float().cpu(), xr.grad, "dqkv"), (tq.grad.cpu(), tr.grad, "dtable")):
        l2 = ((got - want).norm() / want.norm()).item()
        cos = (got.flatten() @ want.flatten() / (got.norm() * want.norm())).item()
        assert l2 < 3e-2 and cos > 0.999, (nm, l2, cos)


def _setup(cfg, B, T, HW, seed=0):
    from vclip_amd.swin3d import Swin3d
    sd = make_swin3d_weights(cfg, seed=seed)
    m = Swin3d({k: v for k, v in cfg.items() if k != "num_classes"}, num_classes=cfg["num_classes"])
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    m.stochastic_depth = False
    video = make_synthetic_video(B, T, HW, seed=1)
    labels = np.random.RandomState(2).randint(0, 2, size=B)
    return m, sd, torch.from_numpy(video), torch.from_numpy(labels).long()


def _compare(model, ref_grads, l2_tol=5e-2, cos_tol=0.998):
    worst = []
    for n in model.state_dict():
        g = model.P(n).grad
        assert g is not None, n
        g = g.detach().cpu().double().reshape(-1)
        r = ref_grads[n].double().reshape(-1)
        if n.endswith("qkv.bias"):  # key third: softmax is invariant to a key bias (exact-zero gradient)
            D = r.numel() // 3
            scale = ref_grads[n.replace("bias", "weight")].double().norm()
            assert g[D:2 * D].norm() < 1e-2 * scale, n
            g, r = torch.cat([g[:D], g[2 * D:]]), torch.cat([r[:D], r[2 * D:]])
        if r.norm() < 1e-12:
            assert g.norm() < 1e-6, n
            continue
        l2 = float((g - r).norm() / r.norm())
        cos = float(g @ r / (g.norm() * r.norm()))
        worst.append((l2, n, cos))
        assert l2 < l2_tol and cos > cos_tol, (n, l2, cos)
    return max(worst)


@pytest.mark.parametrize("cfg,B,T,HW", [(TINY, 2, 8, 24), (STAGE1, 1, 16, 56)], ids=["tiny-B2", "stage1-B1"])
def test_train_gradients_match_autograd(cfg, B, T, HW):
    model, sd, video, labels = _setup(cfg, B, T, HW)
    logits = model(video.to(DEV))
    loss = torch.nn.functional.cross_entropy(logits, labels.to(DEV))
    loss.backward()
    p = {k: torch.from_numpy(v).clone().requires_grad_() for k, v in sd.items()}
    rl = ref.swin3d_forward(p, cfg, video)
    rloss = torch.nn.functional.cross_entropy(rl, labels)
    rloss.backward()
    np.testing.assert_allclose(logits.detach().cpu().numpy(), rl.detach().numpy(), rtol=0, atol=1e-2)
    assert abs(float(loss) - float(rloss)) < 1e-2
    print("worst gradient (rel L2, name, cos):", _compare(model, {k: v.grad for k, v in p.items()}))


def test_train_logits_equal_inference_logits():
    model, sd, video, labels = _setup(TINY, 2, 8, 24)
    x = video.to(DEV)
    tr = model(x).detach()
    model.eval()
    with torch.no_grad():
        ev = model(x)
    torch.testing.assert_close(tr, ev, rtol=0, atol=5e-3)


def test_stochastic_depth_drops_whole_clips():
    """torchvision StochasticDepth(p, "row"): at p = 0 the train logits equal the deterministic ones
    bit for bit; at p > 0 the per-clip keep masks come from torch's RNG (same seed, same logits)."""
    model, sd, video, labels = _setup(TINY, 2, 8, 24)
    x = video.to(DEV)
    model.stochastic_depth = True
    model.cfg["stochastic_depth_prob"] = 0.0
    a = model(x).detach()
    model.stochastic_depth = False
    b = model(x).detach()
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    model.stochastic_depth = True
    model.cfg["stochastic_depth_prob"] = 0.5
    torch.manual_seed(0)
    c1 = model(x).detach()
    torch.manual_seed(0)
    c2 = model(x).detach()
    torch.testing.assert_close(c1, c2, rtol=0, atol=0)  # the masks come from torch's (seeded) RNG


def test_reference_training_loop_with_adamw():
    from vclip_amd.optim import AdamW
    model, sd, video, labels = _setup(TINY, 2, 8, 24)
    opt = AdamW(model.parameters(), lr=1e-3, weight_decay=0.05)
    p = {k: torch.from_numpy(v).clone().requires_grad_() for k, v in sd.items()}
    ropt = torch.optim.AdamW(list(p.values()), lr=1e-3, weight_decay=0.05)
    crit = torch.nn.CrossEntropyLoss()
    losses, rlosses = [], []
    for _ in range(3):
        opt.zero_grad()
        loss = crit(model(video.to(DEV)), labels.to(DEV))
        loss.backward()
        opt.step()
        losses.append(float(loss))
        ropt.zero_grad()
        rl = crit(ref.swin3d_forward(p, TINY, video), labels)
        rl.backward()
        ropt.step()
        rlosses.append(float(rl))
    np.testing.assert_allclose(losses, rlosses, rtol=0, atol=2e-2)
    model.eval()  # eval after training sees the updated masters (inference pack refreshed)
    with torch.no_grad():
        ev = model(video.to(DEV)).cpu()
        rv = ref.swin3d_forward({k: v.cpu() for k, v in model.state_dict().items()}, TINY, video)
    np.testing.assert_allclose(ev.numpy(), rv.numpy(), rtol=0, atol=1e-2)
