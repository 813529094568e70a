"""GPU parity tests of the train-step kernels through the C-ABI
(vclip_amd.ops), each against torch fp32 autograd of the same op on the same bf16-rounded
inputs — the arithmetic the reference's `loss.backward()` / `optimizer.step()` run
(vivit_transformer/vivit_classifier/trainers/trainer.py:145-146).

Tolerances (stated per test): fp32-accumulated reductions ~1e-5 relative; bf16 MFMA
products (attention backward, weight gradients) 1-2e-2 relative to the tensor's scale.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
LN2 = math.log(2.0)


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vclip_amd import _lib as L
    L.load()


def ops():
    from vclip_amd import ops as O
    return O


def rel_err(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    return float((got - ref).norm() / ref.norm().clamp_min(1e-30)), float((got - ref).abs().max() / ref.abs().max())


# ------------------------------------------------------------------------- attention backward
def _attn_case(B, S, H, seed):
    g = torch.Generator().manual_seed(seed)
    rows = (B - 1) * S + (S + 63) // 64 * 64 + 64
    q = (torch.randn(B, S, H, 64, generator=g) * 0.4).bfloat16()
    k = torch.randn(B, S, H, 64, generator=g).bfloat16()
    v = torch.randn(B, S, H, 64, generator=g).bfloat16()
    do = (torch.randn(B, S, H, 64, generator=g) * 0.1).bfloat16()
    qkv = torch.zeros(rows, 3 * H * 64, dtype=torch.bfloat16)
    qkv[:B * S, :H * 64] = q.reshape(B * S, -1)
    qkv[:B * S, H * 64:2 * H * 64] = k.reshape(B * S, -1)
    qkv[:B * S, 2 * H * 64:] = v.reshape(B * S, -1)
    dout = torch.zeros(rows, H * 64, dtype=torch.bfloat16)
    dout[:B * S] = do.reshape(B * S, -1)
    return q, k, v, do, qkv, dout, rows


def _attn_ref(q, k, v, do):
    """log2-domain softmax attention (q holds q' = q*scale*log2 e): P = softmax(ln2 * q'k^T)."""
    qf, kf, vf = (t.float().permute(0, 2, 1, 3).requires_grad_() for t in (q, k, v))
    p = torch.softmax((qf @ kf.transpose(-1, -2)) * LN2, dim=-1)
    o = p @ vf
    lse2 = torch.logsumexp((qf @ kf.transpose(-1, -2)) * LN2, dim=-1) / LN2
    o.backward(do.float().permute(0, 2, 1, 3))
    return o.detach(), lse2.detach(), qf.grad, kf.grad, vf.grad


@pytest.mark.parametrize("B,S,H", [(1, 64, 1), (2, 65, 2), (2, 197, 2), (1, 300, 3), (2, 130, 1)])
def test_attention_fwd_lse_bwd(B, S, H):
    O = ops()
    q, k, v, do, qkv, dout, rows = _attn_case(B, S, H, seed=S * 10 + B)
    o_ref, lse_ref, dq_ref, dk_ref, dv_ref = _attn_ref(q, k, v, do)
    qkv_d, dout_d = qkv.to(DEV), dout.to(DEV)
    out = torch.zeros(rows, H * 64, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B * H * S, dtype=torch.float32, device=DEV)
    O.attention_fwd_lse(qkv_d, B, S, H, out, lse)
    o_got = out[:B * S].float().cpu().reshape(B, S, H, 64).permute(0, 2, 1, 3)
    assert rel_err(o_got, o_ref)[1] < 2e-2
    # lse: base-2 log-sum-exp of the scores, per (clip, head, query)
    np.testing.assert_allclose(lse.cpu().reshape(B, H, S).numpy(), lse_ref.numpy(), rtol=0, atol=2e-3)
    delta = torch.zeros(B * H * S, dtype=torch.float32, device=DEV)
    dqkv = torch.zeros(rows, 3 * H * 64, dtype=torch.bfloat16, device=DEV)
    O.attention_bwd(qkv_d, out, dout_d, lse, delta, B, S, H, dqkv)
    got = dqkv[:B * S].float().cpu().reshape(B, S, 3, H, 64)
    for i, ref in enumerate((dq_ref, dk_ref, dv_ref)):
        g = got[:, :, i].permute(0, 2, 1, 3)
        l2, mx = rel_err(g, ref)
        assert l2 < 1.5e-2 and mx < 3e-2, ("qkv"[i], l2, mx)
    # padding rows past the last clip are never written
    assert dqkv[B * S:].abs().sum().item() == 0


def test_attention_bwd_vivit_size():
    """ViViT-B/16x2 geometry (S = 3137, 12 heads), one clip: the multi-tile pipeline with a partial last tile."""
    O = ops()
    B, S, H = 1, 3137, 12
    q, k, v, do, qkv, dout, rows = _attn_case(B, S, H, seed=3137)
    o_ref, lse_ref, dq_ref, dk_ref, dv_ref = _attn_ref(q, k, v, do)
    qkv_d, dout_d = qkv.to(DEV), dout.to(DEV)
    out = torch.zeros(rows, H * 64, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B * H * S, dtype=torch.float32, device=DEV)
    delta = torch.zeros_like(lse)
    dqkv = torch.zeros(rows, 3 * H * 64, dtype=torch.bfloat16, device=DEV)
    O.attention_fwd_lse(qkv_d, B, S, H, out, lse)
    O.attention_bwd(qkv_d, out, dout_d, lse, delta, B, S, H, dqkv)
    got = dqkv[:B * S].float().cpu().reshape(B, S, 3, H, 64)
    for i, ref in enumerate((dq_ref, dk_ref, dv_ref)):
        l2, mx = rel_err(got[:, :, i].permute(0, 2, 1, 3), ref)
        assert l2 < 1.5e-2 and mx < 3e-2, ("qkv"[i], l2, mx)


# ------------------------------------------------------------------------- LayerNorm backward
@pytest.mark.parametrize("M,D", [(5, 768), (3137 * 2, 768), (100, 256), (37, 1024)])
def test_layernorm_bwd(M, D):
    O = ops()
    g = torch.Generator().manual_seed(M + D)
    x = torch.randn(M, D, generator=g) * 2 + 0.5
    dy = torch.randn(M, D, generator=g)
    gamma = 1 + 0.1 * torch.randn(D, generator=g)
    beta = 0.1 * torch.randn(D, generator=g)
    dx0 = torch.randn(M, D, generator=g)
    xr = x.clone().requires_grad_()
    gr, br = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-6).backward(dy)
    dx = dx0.to(DEV).clone()
    dxb = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    dg = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    nb = min(512, (M + 3) // 4)
    work = torch.empty((nb + (nb + 31) // 32) * 4 * D, device=DEV)
    s_in, s_out = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    O.layernorm_bwd(dy.to(DEV), x.to(DEV), gamma.to(DEV), 1e-6, dx, dxb, dg, db, work, dsum_in=s_in, dsum_out=s_out)
    ref = dx0 + xr.grad
    np.testing.assert_allclose(dx.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    # the fused bias gradients: column sums of dx before and after the update
    np.testing.assert_allclose(s_in.cpu().numpy(), dx0.double().sum(0).numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(s_out.cpu().numpy(), ref.double().sum(0).numpy(), rtol=1e-4, atol=1e-3)
    # without the sums (the layernorm_before call of the train step)
    dx2 = dx0.to(DEV).clone()
    O.layernorm_bwd(dy.to(DEV), x.to(DEV), gamma.to(DEV), 1e-6, dx2, dxb, dg, db, work)
    torch.testing.assert_close(dx2, dx)
    np.testing.assert_array_equal(dxb.cpu().float().numpy(), dx.cpu().bfloat16().float().numpy())
    np.testing.assert_allclose(dg.cpu().numpy(), gr.grad.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(db.cpu().numpy(), br.grad.numpy(), rtol=1e-4, atol=1e-3)


# ------------------------------------------------------------------------- column sums / bias grads
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("R,N", [(1, 768), (12800, 3072), (257, 130)])
def test_colsum(dtype, R, N):
    O = ops()
    g = torch.Generator().manual_seed(R + N)
    x = torch.randn(R, N, generator=g).to(dtype)
    out = torch.zeros(N, device=DEV)
    work = torch.empty(256 * N, device=DEV)
    O.colsum(x.to(DEV), out, work, nscaled=N // 3, scale=0.5)
    ref = x.double().sum(0)
    ref[:N // 3] *= 0.5
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), rtol=1e-5, atol=1e-4 * math.sqrt(R))


@pytest.mark.parametrize("R,N", [(12800, 3072), (12800, 2304), (1000, 520)])
def test_colsum_bf16_vector_pass_bit_identical(R, N):
    """The 16-B-per-lane bf16 first pass (aligned rows, N % 8 == 0) keeps the 2-B pass's summation
    order per column: the same input through a row stride that is not a multiple of 8 (the 2-B pass)
    gives the same bits."""
    O = ops()
    g = torch.Generator().manual_seed(R * 7 + N)
    x = torch.randn(R, N, generator=g).to(torch.bfloat16)
    xa = x.to(DEV)
    xs = torch.zeros(R, N + 1, dtype=torch.bfloat16, device=DEV)
    xs[:, :N] = xa
    outs = []
    for src in (xa, xs[:, :N]):
        out = torch.zeros(N, device=DEV)
        O.colsum(src, out, torch.empty(256 * N, device=DEV), nscaled=N // 3, scale=0.5)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])


# ------------------------------------------------------------------------- weight gradient GEMM
@pytest.mark.parametrize("M,N1,N2,split", [(256, 128, 128, False), (12800, 768, 768, True), (4096, 2304, 768, True),
                                           (12800, 768, 3072, True), (3200, 3072, 768, False), (6272, 768, 1536, True),
                                           (2080, 256, 512, True), (64, 512, 256, True),
                                           # the 128 x 128 kernel (N1 or N2 not a multiple of 256)
                                           (3136, 384, 128, True), (12544, 128, 384, True), (1024, 640, 384, False)])
def test_wgrad(M, N1, N2, split):
    O = ops()
    g = torch.Generator().manual_seed(M + N1 + N2)
    gg = torch.randn(M, N1 + 64, generator=g).bfloat16()[:, :N1]  # row stride > N1
    xx = torch.randn(M, N2, generator=g).bfloat16()
    out = torch.zeros(N1, N2, device=DEV)
    work = torch.empty(64 * N1 * N2, device=DEV) if split else None
    c = 0.125 * 1.4426950408889634
    O.wgrad(gg.to(DEV), xx.to(DEV), out, work, nscaled=N1 // 3, scale=c)
    ref = gg.double().T @ xx.double()
    ref[:N1 // 3] *= c
    l2, mx = rel_err(out, ref)
    assert l2 < 1e-5 and mx < 1e-4, (l2, mx)


# ------------------------------------------------------------------------- GEMM training epilogues
def test_gemm_training_epilogues():
    O = ops()
    g = torch.Generator().manual_seed(5)
    M, N, K = 512, 384, 256
    a = (torch.randn(M, K, generator=g) * 0.5).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, generator=g) * 0.1
    acc = a.double() @ w.double().T + bias.double()
    ad, wd, bd = a.to(DEV), w.to(DEV), bias.to(DEV)
    # residual into a new buffer
    res = torch.randn(M, N, generator=g)
    out = torch.zeros(M, N, device=DEV)
    O.gemm(ad, wd, bd, "bias_add_f32", out, aux=res.to(DEV))
    np.testing.assert_allclose(out.cpu().double().numpy(), (acc + res.double()).numpy(), rtol=0, atol=2e-4)
    # gelu with the pre-activation saved
    h = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    pre = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    O.gemm(ad, wd, bd, "bias_gelu_tanh_save", h, aux=pre)
    np.testing.assert_allclose(pre.cpu().float().numpy(), acc.float().bfloat16().float().numpy(), rtol=0, atol=1.6e-2)
    from oracle.vivit_ref import gelu_fast
    np.testing.assert_allclose(h.cpu().float().numpy(), gelu_fast(acc.float()).numpy(), rtol=1e-2, atol=1e-2)
    # gelu backward fused into the dgrad epilogue
    dh = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    O.gemm(ad, wd, bd, "dgelu_tanh", dh, aux=pre)
    p = pre.cpu().float().requires_grad_()
    gelu_fast(p).backward(torch.ones_like(p))
    ref = acc.float() * p.grad
    np.testing.assert_allclose(dh.cpu().float().numpy(), ref.numpy(), rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("cfg", [4, 5, -1])
def test_gemm_gelu_save_configs(cfg):
    """GELU_SAVE on the persistent 256x256 kernel (cfg 4, two bf16 outputs per tile) and cfg 5:
    identical bits (same fp32 accumulation order per output is not guaranteed, so compare to the
    double reference), at a shape with several tiles per workgroup."""
    O = ops()
    g = torch.Generator().manual_seed(6)
    M, N, K = 4096, 3072, 768
    a = (torch.randn(M, K, generator=g) * 0.5).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, generator=g) * 0.1
    acc = (a.double() @ w.double().T + bias.double()).float()
    h = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    pre = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    O.gemm(a.to(DEV), w.to(DEV), bias.to(DEV), "bias_gelu_tanh_save", h, aux=pre, cfg=cfg)
    np.testing.assert_allclose(pre.cpu().float().numpy(), acc.bfloat16().float().numpy(), rtol=0, atol=1.6e-2)
    from oracle.vivit_ref import gelu_fast
    np.testing.assert_allclose(h.cpu().float().numpy(), gelu_fast(acc).numpy(), rtol=1e-2, atol=1e-2)


# ------------------------------------------------------------------------- classifier head / embeddings
def test_cls_head_bwd():
    O = ops()
    g = torch.Generator().manual_seed(11)
    B, S, D, nl = 3, 17, 768, 2
    x = torch.randn(B * S + 5, D, generator=g)
    gamma = 1 + 0.1 * torch.randn(D, generator=g)
    beta = 0.1 * torch.randn(D, generator=g)
    wc = 0.02 * torch.randn(nl, D, generator=g)
    dl = torch.randn(B, nl, generator=g)
    xr = x.clone().requires_grad_()
    gr, br, wr = gamma.clone().requires_grad_(), beta.clone().requires_grad_(), wc.clone().requires_grad_()
    bcr = torch.zeros(nl, requires_grad=True)
    y = torch.nn.functional.layer_norm(xr[0:B * S:S], (D,), gr, br, 1e-6)
    (y @ wr.T + bcr).backward(dl)
    dx = torch.zeros(B * S + 5, D, device=DEV)
    dxb = torch.zeros(B * S + 5, D, dtype=torch.bfloat16, device=DEV)
    dwc, dbc = torch.zeros(nl, D, device=DEV), torch.zeros(nl, device=DEV)
    dg, db = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    O.cls_head_bwd(x.to(DEV), B, S, gamma.to(DEV), beta.to(DEV), 1e-6, wc.to(DEV), dl.to(DEV), dx, dxb, dwc, dbc, dg, db)
    for got, ref in ((dx, xr.grad), (dwc, wr.grad), (dbc, bcr.grad), (dg, gr.grad), (db, br.grad)):
        np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)


def test_embed_bwd():
    O = ops()
    g = torch.Generator().manual_seed(12)
    B, S, D = 3, 50, 768
    dx = torch.randn(B * S + 7, D, generator=g)
    dpos = torch.zeros(S * D, device=DEV)
    dcls = torch.zeros(D, device=DEV)
    demb = torch.zeros(B * (S - 1) + 3, D, dtype=torch.bfloat16, device=DEV)
    O.embed_bwd(dx.to(DEV), B, S, dpos, dcls, demb)
    v = dx[:B * S].reshape(B, S, D)
    np.testing.assert_allclose(dpos.cpu().reshape(S, D).numpy(), v.sum(0).numpy(), rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(dcls.cpu().numpy(), v[:, 0].sum(0).numpy(), rtol=1e-6, atol=1e-5)
    np.testing.assert_array_equal(demb[:B * (S - 1)].cpu().float().numpy(),
                                  v[:, 1:].reshape(-1, D).bfloat16().float().numpy())


# ------------------------------------------------------------------------- optimizer / packing
def test_adamw_matches_torch():
    O = ops()
    g = torch.Generator().manual_seed(13)
    n = 100_003
    p0 = torch.randn(n, generator=g)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=0.01)
    p, m, v = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for step in range(1, 4):
        grad = torch.randn(n, generator=g)
        ref.grad = grad.clone()
        opt.step()
        O.adamw(p, (grad * 2).to(DEV), m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, grad_scale=0.5)
    np.testing.assert_allclose(p.cpu().numpy(), ref.detach().numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("N,K,ns", [(200, 132, 70), (2304, 768, 768), (68, 4, 0)])
def test_pack_weight(N, K, ns):
    O = ops()
    g = torch.Generator().manual_seed(14)
    w = torch.randn(N, K, generator=g)
    dst = torch.zeros(N, K, dtype=torch.bfloat16, device=DEV)
    dst_t = torch.zeros(K, N, dtype=torch.bfloat16, device=DEV)
    O.pack_weight(w.to(DEV), dst, dst_t, nscaled=ns, scale=0.3)
    ref = w.clone()
    ref[:ns] *= 0.3
    np.testing.assert_array_equal(dst.cpu().float().numpy(), ref.bfloat16().float().numpy())
    np.testing.assert_array_equal(dst_t.cpu().float().numpy(), ref.T.bfloat16().float().numpy())


def test_adamw_multi_matches_per_tensor():
    """One multi-tensor launch (vc_adamw_multi) = vc_adamw per tensor, bit for bit, over sizes that
    straddle the 1024-element chunks (1, 1023, 1024, 1025, a weight matrix)."""
    O = ops()
    g = torch.Generator(device=DEV).manual_seed(5)
    sizes = [1, 1023, 1024, 1025, 768 * 3072, 7, 4096 + 3]
    mk = lambda n: torch.randn(n, device=DEV, generator=g)  # noqa: E731
    ps, gs = [mk(n) for n in sizes], [mk(n) for n in sizes]
    ms, vs = [mk(n) * 0.1 for n in sizes], [mk(n).abs() * 0.01 for n in sizes]
    ref = [(p.clone(), m.clone(), v.clone()) for p, m, v in zip(ps, ms, vs)]
    for (p, m, v), gr in zip(ref, gs):
        O.adamw(p, gr, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3, 0.5)
    O.adamw_multi(ps, gs, ms, vs, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3, 0.5)
    torch.cuda.synchronize()
    for (rp, rm, rv), p, m, v in zip(ref, ps, ms, vs):
        assert torch.equal(p, rp) and torch.equal(m, rm) and torch.equal(v, rv)


def test_wgrad_pp_bit_identical_to_big(tmp_path):
    """The ping-pong weight-gradient kernel (wgrad_pp_kernel, the default) runs wgrad_big_kernel's MFMA
    chain per output: a child process with VCLIP_WGRAD_PP=0 (the big kernel) must give the same bits,
    with and without split-K partials."""
    import subprocess
    import sys
    O = ops()
    g = torch.Generator().manual_seed(11)
    cases = [(12800, 768, 3072, True), (3200, 2304, 768, False), (4096, 768, 768, True)]
    data = {}
    for i, (M, N1, N2, split) in enumerate(cases):
        gg = torch.randn(M, N1, generator=g).bfloat16()
        xx = torch.randn(M, N2, generator=g).bfloat16()
        out = torch.zeros(N1, N2, device=DEV)
        work = torch.empty(4 * N1 * N2, device=DEV) if split else None
        O.wgrad(gg.to(DEV), xx.to(DEV), out, work, nscaled=N1 // 3, scale=0.3)
        data[f"g{i}"], data[f"x{i}"], data[f"o{i}"] = gg, xx, out.cpu()
    torch.save(data, tmp_path / "in.pt")
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    code = (
        "import sys, torch; sys.path.insert(0, %r)\n"
        "from vclip_amd import ops as O\n"
        "d = torch.load(%r, weights_only=True); r = {}\n"
        "for i, (M, N1, N2, split) in enumerate(%r):\n"
        "    out = torch.zeros(N1, N2, device='cuda')\n"
        "    work = torch.empty(4 * N1 * N2, device='cuda') if split else None\n"
        "    O.wgrad(d[f'g{i}'].cuda(), d[f'x{i}'].cuda(), out, work, nscaled=N1 // 3, scale=0.3)\n"
        "    r[f'o{i}'] = out.cpu()\n"
        "torch.save(r, %r)\n" % (root, str(tmp_path / "in.pt"), cases, str(tmp_path / "out.pt")))
    env = dict(__import__("os").environ, VCLIP_WGRAD_PP="0")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    big = torch.load(tmp_path / "out.pt", weights_only=True)
    for i in range(len(cases)):
        assert torch.equal(data[f"o{i}"], big[f"o{i}"]), i
