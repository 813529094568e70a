"""TimeSformer train step (the TimeSformer folder's main.py trains by default:
timesformer/timesformer_classifier/trainers/trainer.py:139-174 — zero_grad, model(**inputs),
CrossEntropyLoss, loss.backward(), AdamW.step()) on the HIP autograd ops (vclip_amd/autograd_ops.py),
against fp32 torch autograd of oracle/timesformer_ref.py (pinned to HF TimeSformer goldens).

Tolerances as the ViViT train tests: bf16 operands with fp32 accumulation, so per-parameter
gradients by relative L2 (<= 5e-2) and cosine (>= 0.998); logits 1e-2 absolute; AdamW trajectories
by the relative error of each tensor's accumulated update (<= 0.1)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
SMALL = dict(image_size=32, patch_size=16, num_channels=3, num_frames=4, hidden_size=256, num_hidden_layers=2,
             num_attention_heads=4, intermediate_size=512, hidden_act="gelu", layer_norm_eps=1e-6)
# TimeSformer-B per-layer geometry (224^2, 196 patches, 8 frames, D 768, 12 heads), one layer
WIDE = dict(SMALL, image_size=224, num_frames=8, hidden_size=768, num_attention_heads=12, intermediate_size=3072,
            num_hidden_layers=1)


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vclip_amd import _lib as L
    L.load()


def _setup(cfg, B, seed=0):
    from vclip_amd.timesformer import TimesformerConfig, TimesformerForVideoClassification
    from vclip_amd.weights import make_synthetic_clips, make_timesformer_weights
    c = TimesformerConfig(**cfg, id2label={0: "non-referral", 1: "referral"})
    sd = make_timesformer_weights(c.as_shape_cfg(), seed=seed)
    pix = make_synthetic_clips(B, cfg["num_frames"], cfg["image_size"], seed=1)
    labels = np.random.RandomState(2).randint(0, 2, size=B)
    model = TimesformerForVideoClassification(c)
    model.load_state_dict(sd)
    model = model.to(DEV).train()
    return model, sd, torch.from_numpy(pix), torch.from_numpy(labels).long(), c


def _ref_cfg(c):
    return dict(c.as_shape_cfg(), num_attention_heads=c.num_attention_heads, layer_norm_eps=c.layer_norm_eps)


def _oracle(sd, c, pix, labels):
    from oracle.timesformer_ref import timesformer_forward
    ref = {k: torch.from_numpy(v).clone().requires_grad_() for k, v in sd.items()}
    logits = timesformer_forward(ref, _ref_cfg(c), pix)
    loss = torch.nn.functional.cross_entropy(logits, labels)
    loss.backward()
    return float(loss), logits.detach(), {k: v.grad for k, v in ref.items()}


def _compare(model, ref_grads, l2_tol=5e-2, cos_tol=0.998):
    worst = []
    for n, p in model.state_dict().items():
        g = model.P(n).grad
        assert g is not None, n
        g = g.detach().cpu().double().reshape(-1)
        r = ref_grads[n].double().reshape(-1)
        if n.endswith("qkv.bias"):
            # the key third of the qkv bias has an exact-zero gradient (softmax is invariant to a
            # key bias); compare the query and value thirds, bound the key third by the weight's scale
            D = r.numel() // 3
            scale = ref_grads[n.replace("bias", "weight")].double().norm()
            assert g[D:2 * D].norm() < 1e-2 * scale and r[D:2 * D].norm() < 1e-2 * scale, n
            g = torch.cat([g[:D], g[2 * D:]])
            r = torch.cat([r[:D], r[2 * D:]])
        if r.norm() < 1e-12:
            assert g.norm() < 1e-6, n
            continue
        l2 = float((g - r).norm() / r.norm())
        cos = float(g @ r / (g.norm() * r.norm()))
        worst.append((l2, n, cos))
        assert l2 < l2_tol and cos > cos_tol, (n, l2, cos)
    return max(worst)


@pytest.mark.parametrize("cfg,B", [(SMALL, 2), (SMALL, 3), (WIDE, 1)], ids=["small-B2", "small-B3", "wide-B1"])
def test_train_gradients_match_autograd(cfg, B):
    model, sd, pix, labels, c = _setup(cfg, B)
    out = model(pixel_values=pix.to(DEV))
    loss = torch.nn.functional.cross_entropy(out.logits, labels.to(DEV))
    loss.backward()
    ref_loss, ref_logits, ref_grads = _oracle(sd, c, pix, labels)
    np.testing.assert_allclose(out.logits.detach().cpu().numpy(), ref_logits.numpy(), rtol=0, atol=1e-2)
    assert abs(float(loss) - ref_loss) < 1e-2
    print("worst gradient (rel L2, name, cos):", _compare(model, ref_grads))


def test_train_logits_equal_inference_logits():
    """The autograd train forward and the fused inference forward are the same model."""
    model, sd, pix, labels, c = _setup(SMALL, 2)
    x = pix.to(DEV)
    tr = model(pixel_values=x).logits.detach()
    model.eval()
    with torch.no_grad():
        ev = model(pixel_values=x).logits
    torch.testing.assert_close(tr, ev, rtol=0, atol=5e-3)


def test_reference_training_loop_with_adamw():
    """Three steps of the reference loop: vclip AdamW on the HIP model vs torch AdamW on the oracle."""
    from oracle.timesformer_ref import timesformer_forward
    from vclip_amd.optim import AdamW
    model, sd, pix, labels, c = _setup(SMALL, 2)
    opt = AdamW(model.parameters(), lr=1e-3, weight_decay=0.01)
    ref = {k: torch.from_numpy(v).clone().requires_grad_() for k, v in sd.items()}
    ropt = torch.optim.AdamW(list(ref.values()), lr=1e-3, weight_decay=0.01)
    crit = torch.nn.CrossEntropyLoss()
    losses, rlosses = [], []
    for _ in range(3):
        opt.zero_grad()
        loss = crit(model(pixel_values=pix.to(DEV)).logits, labels.to(DEV))
        loss.backward()
        opt.step()
        losses.append(float(loss))
        ropt.zero_grad()
        rl = crit(timesformer_forward(ref, _ref_cfg(c), pix), labels)
        rl.backward()
        ropt.step()
        rlosses.append(float(rl))
    np.testing.assert_allclose(losses, rlosses, rtol=0, atol=2e-2)
    for n, p in model.state_dict().items():
        du = p.detach().cpu().double() - torch.from_numpy(sd[n]).double()
        dr = ref[n].detach().double() - torch.from_numpy(sd[n]).double()
        if n.endswith("qkv.bias"):  # the key third: exact gradient 0, AdamW steps on rounding noise
            D = du.numel() // 3
            du, dr = torch.cat([du[:D], du[2 * D:]]), torch.cat([dr[:D], dr[2 * D:]])
        e = float((du - dr).abs().mean() / dr.abs().mean().clamp_min(1e-12))
        assert e < 0.1, (n, e)
    model.eval()  # eval after training sees the updated masters (inference pack refreshed)
    with torch.no_grad():
        ev = model(pixel_values=pix.to(DEV)).logits.cpu()
        rv = timesformer_forward({k: v.cpu() for k, v in model.state_dict().items()}, _ref_cfg(c), pix)
    np.testing.assert_allclose(ev.numpy(), rv.numpy(), rtol=0, atol=1e-2)


def test_temporal_attention_backward_vs_autograd():
    """vc_temporal_attention_bwd against torch autograd of the same softmax (base-2 scores of the
    prescaled q'), T in {4, 8, 32}, on the clip layout with CLS rows."""
    from vclip_amd import autograd_ops as A
    for T in (4, 8, 32):
        B, P, H = 2, 3, 2
        S = 1 + P * T
        g = torch.Generator().manual_seed(T)
        qkv = (torch.randn(B * S, 3 * H * 64, generator=g) * 0.5).bfloat16()
        dout = torch.randn(B * S, H * 64, generator=g).bfloat16()
        dout.view(B, S, -1)[:, 0] = 0
        x = qkv.to(DEV).requires_grad_()
        o = A.temporal_attention(x, B, P, T, H)
        o.backward(dout.to(DEV))
        q = qkv.float().view(B, S, 3, H, 64)[:, 1:].reshape(B, P, T, 3, H, 64).requires_grad_()
        s = torch.einsum("bptha,bpuha->bphtu", q[:, :, :, 0], q[:, :, :, 1]) * np.log(2.0)
        ref = torch.einsum("bphtu,bpuha->bptha", torch.softmax(s, -1), q[:, :, :, 2])
        ref.backward(dout.float().view(B, S, H, 64)[:, 1:].reshape(B, P, T, H, 64))
        got = x.grad.float().cpu().view(B, S, 3, H, 64)
        assert (got[:, 0] == 0).all()
        want = q.grad.reshape(B, P * T, 3, H, 64)
        err = (got[:, 1:] - want).abs().max().item()
        assert err < 3e-2 * max(1.0, want.abs().max().item()), (T, err)
        torch.testing.assert_close(o[:, :].float().cpu().view(B, S, H, 64)[:, 1:].reshape(B, P, T, H, 64),
                                   ref.detach(), rtol=0, atol=2e-2)


def test_gelu_erf_forward_backward():
    from vclip_amd import autograd_ops as A
    x = (torch.randn(128, 64) * 3).bfloat16()
    xd = x.to(DEV).requires_grad_()
    y = A.gelu_erf(xd)
    dy = torch.randn(128, 64)
    y.backward(dy.to(DEV).bfloat16())
    xr = x.float().requires_grad_()
    yr = torch.nn.functional.gelu(xr)
    yr.backward(dy.bfloat16().float())
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(xd.grad.float().cpu(), xr.grad, rtol=2e-2, atol=2e-2)
