"""ResNet3D-50 train step (resnet50-3d-video/video_classifier/trainers/trainer.py:106-123:
model.train(), outputs = model(videos), CrossEntropyLoss, loss.backward(), Adam.step()) on the HIP
autograd ops, against fp32 torch autograd of oracle/resnet3d_ref.py in training mode (BatchNorm
with batch statistics; pytorchvideo is absent, so parity with the library itself is UNPINNED).

Kernel pieces (col2im, MaxPool3d backward, BatchNorm train forward / backward, the head) are
checked one by one against torch autograd of the same op; the whole step by per-parameter
gradients: bf16 GEMM operands and bf16 activations with fp32 accumulation and fp32 BatchNorm,
so relative L2 <= 6e-2 and cosine >= 0.998; logits 2e-2 absolute.  The head's dropout (random by
design) is switched off for the gradient comparisons and checked separately through its mask."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import resnet3d_ref as ref
from vclip_amd.weights import make_resnet3d_weights, make_synthetic_video

pytestmark = pytest.mark.gpu
DEV = "cuda"

# every structural feature of the 50-layer net (branch1 on each stage, stride 2, (3,1,1) conv_a,
# identity skips) and its channel widths with 6 blocks; 64x64 frames end on a 2x2 map
SMALL = dict(depths=(2, 1, 1, 2), stem_dim=64, conv_a_kernels=((1, 1, 1), (1, 1, 1), (3, 1, 1), (3, 1, 1)),
             spatial_strides=(1, 2, 2, 2), head_pool=(2, 2, 2), num_classes=2, bn_eps=1e-5)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vclip_amd import _lib
    _lib.load()


def _cl(x):
    """[B, C, T, H, W] -> channels-last rows [B*T*H*W, C]."""
    return x.permute(0, 2, 3, 4, 1).reshape(-1, x.shape[1])


@pytest.mark.parametrize("kernel,stride,pad,C", [((1, 3, 3), (1, 2, 2), (0, 1, 1), 64), ((3, 1, 1), (1, 1, 1), (1, 0, 0), 16),
                                                  ((1, 1, 1), (1, 2, 2), (0, 0, 0), 32), ((1, 3, 3), (1, 1, 1), (0, 1, 1), 8)])
def test_col2im_is_im2col_adjoint(kernel, stride, pad, C):
    from vclip_amd import autograd_ops as A
    B, T, H, W = 2, 4, 9, 11
    g = torch.Generator().manual_seed(C)
    x = torch.randn(B * T * H * W, C, generator=g).bfloat16()
    xd = x.to(DEV).requires_grad_()
    a = A.im2col_cl(xd, B, (T, H, W), C, kernel, stride, pad)
    da = torch.randn(a.shape, generator=g).bfloat16()
    a.backward(da.to(DEV))
    # torch: the same patches by unfold over the channels-last view, columns (kt, kh, kw, c)
    xr = x.float().requires_grad_()
    v = xr.view(B, T, H, W, C).permute(0, 4, 1, 2, 3)
    v = F.pad(v, (pad[2], pad[2], pad[1], pad[1], pad[0], pad[0]))
    u = v.unfold(2, kernel[0], stride[0]).unfold(3, kernel[1], stride[1]).unfold(4, kernel[2], stride[2])
    ar = u.permute(0, 2, 3, 4, 5, 6, 7, 1).reshape(a.shape[0], -1)
    assert torch.equal(a.cpu(), ar.detach().bfloat16())
    ar.backward(da.float())
    torch.testing.assert_close(xd.grad.float().cpu(), xr.grad.bfloat16().float(), rtol=1e-2, atol=1e-2)


def test_maxpool_backward_first_max():
    from vclip_amd import autograd_ops as A
    B, C, T, H, W = 2, 32, 3, 17, 15
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, C, T, H, W, generator=g).bfloat16().float()
    x[0, :, 1, 4:8, 4:8] = 0.5  # ties: the gradient goes to the first maximum in scan order
    xd = _cl(x).bfloat16().to(DEV).requires_grad_()
    y = A.maxpool(xd, B, (T, H, W), C, (1, 3, 3), (1, 2, 2), (0, 1, 1))
    xr = x.clone().requires_grad_()
    yr = F.max_pool3d(xr, (1, 3, 3), (1, 2, 2), (0, 1, 1))
    assert torch.equal(y.float().cpu(), _cl(yr.detach()))
    dy = torch.randn(yr.shape, generator=g).bfloat16().float()
    yr.backward(dy)
    y.backward(_cl(dy).bfloat16().to(DEV))
    torch.testing.assert_close(xd.grad.float().cpu(), _cl(xr.grad).bfloat16().float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,C,relu,res", [(3000, 64, True, False), (50000, 256, True, True), (777, 128, False, False),
                                          (4096, 2048, True, True)])
def test_batchnorm_train_forward_backward(M, C, relu, res):
    from vclip_amd import autograd_ops as A
    g = torch.Generator().manual_seed(M + C)
    y = torch.randn(M, C, generator=g) * 3 + 1.5
    gamma, beta = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    r = torch.randn(M, C, generator=g).bfloat16() if res else None
    rm, rv = 0.1 * torch.randn(C, generator=g), 1 + torch.rand(C, generator=g)
    dz = torch.randn(M, C, generator=g)
    yd, gd, bd = (t.to(DEV).requires_grad_() for t in (y, gamma, beta))
    rd = r.to(DEV).requires_grad_() if res else None
    rmd, rvd = rm.to(DEV), rv.to(DEV)
    z = A.batchnorm(yd, gd, bd, rmd, rvd, res=rd, relu=relu)
    z.backward(dz.to(DEV))
    yr, gr, br = (t.clone().requires_grad_() for t in (y, gamma, beta))
    rr = r.float().requires_grad_() if res else None
    rmr, rvr = rm.clone(), rv.clone()
    zr = F.batch_norm(yr, rmr, rvr, gr, br, training=True, momentum=0.1, eps=1e-5)
    if res:
        zr = zr + rr
    if relu:
        zr = F.relu(zr)
    zr.backward(dz * (z.cpu().float() != 0) if relu else dz)  # the same ReLU mask (bf16 z rounds some tiny z to 0)
    torch.testing.assert_close(z.float().cpu(), zr.detach(), rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(rmd.cpu(), rmr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rvd.cpu(), rvr, rtol=1e-4, atol=1e-5)
    for got, want in ((yd.grad, yr.grad), (gd.grad, gr.grad), (bd.grad, br.grad)) + \
            (((rd.grad, rr.grad),) if res else ()):
        got = got.float().cpu()
        l2 = float((got - want).norm() / want.norm())
        assert l2 < 1e-2, l2


def test_head_train_matches_torch():
    from vclip_amd import autograd_ops as A
    B, T, HW, C, pt, nl = 3, 6, 4, 256, 4, 2
    g = torch.Generator().manual_seed(9)
    x = torch.randn(B * T * HW, C, generator=g).bfloat16()
    wc, bc = 0.05 * torch.randn(nl, C, generator=g), 0.1 * torch.randn(nl, generator=g)
    keep = torch.bernoulli(torch.full((B, T - pt + 1, C), 0.5), generator=g) * 2
    xd, wd, bd = x.to(DEV).requires_grad_(), wc.to(DEV).requires_grad_(), bc.to(DEV).requires_grad_()
    lo = A.resnet_head(xd, wd, bd, keep.to(DEV), B, T, HW, pt)
    xr, wr, br = x.float().requires_grad_(), wc.clone().requires_grad_(), bc.clone().requires_grad_()
    v = xr.view(B, T, 2, 2, C).permute(0, 4, 1, 2, 3)
    p = F.avg_pool3d(v, (pt, 2, 2), stride=1) * keep.permute(0, 2, 1).reshape(B, C, -1, 1, 1)
    lr = (p.permute(0, 2, 3, 4, 1) @ wr.T + br).mean(dim=(1, 2, 3))
    torch.testing.assert_close(lo.cpu(), lr.detach(), rtol=1e-4, atol=1e-4)
    dl = torch.randn(B, nl, generator=g)
    lo.backward(dl.to(DEV))
    lr.backward(dl)
    for got, want in ((xd.grad, xr.grad), (wd.grad, wr.grad), (bd.grad, br.grad)):
        torch.testing.assert_close(got.float().cpu(), want, rtol=1e-2, atol=1e-5)


def _setup(cfg, B, T, HW, seed=0):
    from vclip_amd.resnet3d import ResNet3d
    sd = make_resnet3d_weights(cfg, seed=seed)
    m = ResNet3d(cfg)
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    m.head_dropout = False
    video = make_synthetic_video(B, T, HW, seed=1)
    labels = np.random.RandomState(2).randint(0, 2, size=B)
    return m, sd, torch.from_numpy(video), torch.from_numpy(labels).long()


def _ref_params(sd):
    return {k: torch.from_numpy(v).clone().requires_grad_(not (k.endswith("running_mean") or k.endswith("running_var")))
            for k, v in sd.items()}


def _grad_errors(grads, p):
    """{name: (rel L2, cos)} of gradients (a model, read through .P(name).grad, or a {name: tensor}
    dict) against the oracle parameters' .grad."""
    out = {}
    for n, q in p.items():
        if not q.requires_grad:
            continue
        g = grads.P(n).grad if hasattr(grads, "P") else grads[n]
        assert g is not None, n
        g = g.detach().cpu().double().reshape(-1)
        r = q.grad.double().reshape(-1)
        out[n] = (float((g - r).norm() / r.norm()), float(g @ r / (g.norm() * r.norm())))
    return out


class _Round(torch.autograd.Function):
    """bf16 storage of a tensor (forward) and / or of its gradient (backward), identity otherwise."""
    @staticmethod
    def forward(ctx, x, fwd: bool, bwd: bool):
        ctx.bwd = bwd
        return x.bfloat16().float() if fwd else x.clone()

    @staticmethod
    def backward(ctx, g):
        return (g.bfloat16().float() if ctx.bwd else g), None, None


# the GPU path's storage precisions on the oracle's graph: activations bf16 (and their gradients,
# autograd's dtype), weights rounded to bf16 for the MFMA (fp32 master gradients), conv outputs fp32
# but their gradients bf16 as the dgrad / wgrad GEMM operands
BF16_STORAGE = {"act": lambda t: _Round.apply(t, True, True), "weight": lambda t: _Round.apply(t, True, False),
                "conv_out": lambda t: _Round.apply(t, False, True)}


@pytest.mark.parametrize("cfg,B,T,HW", [(SMALL, 2, 4, 64), (ref.RESNET3D_50, 2, 4, 224)], ids=["small-B2", "r50-B2-T4"])
def test_train_gradients_match_autograd(cfg, B, T, HW):
    """Train-mode BatchNorm at batch 2 on a random-init net makes the weight gradients ill-conditioned:
    rounding only the WEIGHTS of the fp32 oracle to bf16 already moves them by 10-20% (rel L2).  So
    the bar is set by the precision itself: the fp32 oracle run with this implementation's storage
    precisions (BF16_STORAGE) gives each parameter's attainable error, and the HIP step's gradients
    must stay within that band of the fp32 oracle (<= 1.5x + 0.03 per parameter, medians <= 1.25x +
    0.01), while the well-conditioned head gradients match at 2e-2.  The kernels themselves are checked
    tightly above (col2im, MaxPool, BatchNorm, head) and in test_train_kernels_gpu (GEMMs)."""
    model, sd, video, labels = _setup(cfg, B, T, HW)
    logits = model(video.to(DEV))
    loss = F.cross_entropy(logits, labels.to(DEV))
    loss.backward()
    p = _ref_params(sd)
    rl = ref.resnet3d_forward(p, cfg, video, training=True)
    rloss = F.cross_entropy(rl, labels)
    rloss.backward()
    np.testing.assert_allclose(logits.detach().cpu().numpy(), rl.detach().numpy(), rtol=0, atol=2e-2)
    assert abs(float(loss) - float(rloss)) < 1e-2
    for n, q in p.items():  # the running statistics, updated in place by both
        if not q.requires_grad:
            torch.testing.assert_close(model.P(n).detach().cpu(), q.detach(), rtol=2e-2, atol=2e-2)
    pe = _ref_params(sd)
    F.cross_entropy(ref.resnet3d_forward(pe, cfg, video, training=True, rounding=BF16_STORAGE), labels).backward()
    ours = _grad_errors(model, p)
    band = _grad_errors({n: q.grad for n, q in pe.items() if q.requires_grad}, p)
    for n in ours:
        print(f"{n:55s} ours {ours[n][0]:.4f} (cos {ours[n][1]:.5f})  bf16-storage oracle {band[n][0]:.4f}")
    bad = [(n, ours[n], band[n]) for n in ours if ours[n][0] > 1.5 * band[n][0] + 0.03]
    assert not bad, bad
    med = lambda d: float(np.median([v[0] for v in d.values()]))  # noqa: E731
    assert med(ours) <= 1.25 * med(band) + 0.01, (med(ours), med(band))
    for n in ("blocks.5.proj.weight", "blocks.5.proj.bias"):
        assert ours[n][0] < 2e-2 and ours[n][1] > 0.9998, (n, ours[n])


def test_head_dropout_mask():
    """Dropout(0.5) keep masks come from torch's RNG: seeded runs repeat bit for bit, and the
    logits equal the oracle's with the same mask."""
    model, sd, video, labels = _setup(SMALL, 2, 4, 64)
    model.head_dropout = True
    x = video.to(DEV)
    torch.manual_seed(0)
    a = model(x).detach()
    torch.manual_seed(0)
    b = model(x).detach()
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    model.head_dropout = False
    c = model(x).detach()
    assert (a - c).abs().max() > 1e-4  # the mask changes the logits
    torch.manual_seed(0)
    keep = torch.ones(2, 3, 2048, device=DEV).bernoulli_(0.5).mul_(2.0).cpu()
    rl = ref.resnet3d_forward(_ref_params(sd), SMALL, video, training=True, head_keep=keep).detach()
    np.testing.assert_allclose(a.cpu().numpy(), rl.numpy(), rtol=0, atol=2e-2)


def test_reference_training_loop_with_adam():
    """Three steps of the reference loop with Adam (trainer.py: torch.optim.Adam(lr)) = AdamW with
    weight decay 0; losses against the oracle's trajectory, then eval (BN folded with the updated
    running statistics) against the oracle in eval mode."""
    from vclip_amd.optim import AdamW
    model, sd, video, labels = _setup(SMALL, 2, 4, 64)
    opt = AdamW([q for q in model.parameters() if q.requires_grad], lr=1e-3, weight_decay=0.0)
    p = _ref_params(sd)
    ropt = torch.optim.Adam([q for q in p.values() if q.requires_grad], lr=1e-3)
    crit = torch.nn.CrossEntropyLoss()
    losses, rlosses = [], []
    for _ in range(3):
        opt.zero_grad()
        loss = crit(model(video.to(DEV)), labels.to(DEV))
        loss.backward()
        opt.step()
        losses.append(float(loss))
        ropt.zero_grad()
        rl = crit(ref.resnet3d_forward(p, SMALL, video, training=True), labels)
        rl.backward()
        ropt.step()
        rlosses.append(float(rl))
    np.testing.assert_allclose(losses, rlosses, rtol=0, atol=3e-2)
    model.eval()
    with torch.no_grad():
        ev = model(video.to(DEV)).cpu()
        rv = ref.resnet3d_forward({k: v.cpu() for k, v in model.state_dict().items()}, SMALL, video)
    np.testing.assert_allclose(ev.numpy(), rv.numpy(), rtol=0, atol=2e-2)


def test_train_mode_forward_under_no_grad_keeps_train_semantics():
    """A train-mode forward under torch.no_grad runs the train step's forward as pytorchvideo does:
    batch-statistic BatchNorm (same logits as the grad-enabled forward) and updated running
    statistics; eval mode then runs the folded inference path on those statistics."""
    model, sd, video, labels = _setup(SMALL, 2, 4, 64)
    x = video.to(DEV)
    name = "blocks.1.res_blocks.0.branch2.norm_a.running_mean"
    rm0 = model.state_dict()[name].clone()
    with torch.no_grad():
        lo_ng = model(x)
    rm1 = model.state_dict()[name].clone()
    assert not torch.equal(rm0, rm1)  # running statistics moved
    lo_g = model(x)  # grad-enabled train forward on the same weights: batch statistics again
    torch.testing.assert_close(lo_ng, lo_g.detach(), rtol=0, atol=0)
    model.eval()
    with torch.no_grad():
        lo_eval = model(x)
    assert not torch.allclose(lo_eval, lo_ng)  # running vs batch statistics
