"""3D ResNet-50 on the GPU: conv pieces bit-exact vs torch, end to end vs
oracle/resnet3d_ref.py (fp32 CPU restatement of pytorchvideo create_resnet; pytorchvideo is
not installed, so parity with the library is UNPINNED — SURVEY.md §8c).  bf16 activations
through 16 residual blocks: logits compared at 1e-2 relative to their magnitude (north_star
bf16 tolerance is 1e-2 absolute on O(1) logits; these random-weight logits are O(5))."""
import numpy as np
import pytest
import torch

from oracle import resnet3d_ref as ref
from vclip_amd.weights import make_resnet3d_weights, make_synthetic_video

pytestmark = pytest.mark.gpu
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


def _unfold_ref(x, kernel, stride, pad):
    """x [B,C,T,H,W] -> [B*To*Ho*Wo, C*kvol] with columns (c, kt, kh, kw) (nn.Conv3d weight order)."""
    xp = torch.nn.functional.pad(x, (pad[2], pad[2], pad[1], pad[1], pad[0], pad[0]))
    u = xp.unfold(2, kernel[0], stride[0]).unfold(3, kernel[1], stride[1]).unfold(4, kernel[2], stride[2])
    B, C, To, Ho, Wo = u.shape[:5]
    return u.permute(0, 2, 3, 4, 1, 5, 6, 7).reshape(B * To * Ho * Wo, C * kernel[0] * kernel[1] * kernel[2]), (To, Ho, Wo)


@pytest.mark.parametrize("kernel,stride,pad", [((3, 7, 7), (1, 2, 2), (1, 3, 3)), ((1, 3, 3), (1, 2, 2), (0, 1, 1))])
def test_im2col_ncthw_bit_exact(kernel, stride, pad):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 3, 5, 30, 26, generator=g)
    want, (To, Ho, Wo) = _unfold_ref(x, kernel, stride, pad)
    K = want.shape[1]
    out = torch.zeros(want.shape[0] + 7, (K + 7) // 8 * 8 + 8, dtype=torch.bfloat16, device=DEV)
    ops().conv3d_im2col(x.to(DEV), "ncthw_f32", 2, (5, 30, 26), 3, kernel, stride, pad, out)
    assert torch.equal(out[:want.shape[0], :K].cpu(), want.bfloat16())


@pytest.mark.parametrize("kernel,stride,pad,C", [((1, 3, 3), (1, 2, 2), (0, 1, 1), 64), ((3, 1, 1), (1, 1, 1), (1, 0, 0), 16),
                                                  ((1, 1, 1), (1, 2, 2), (0, 0, 0), 24)])
def test_im2col_channels_last_bit_exact(kernel, stride, pad, C):
    g = torch.Generator().manual_seed(C)
    B, T, H, W = 2, 4, 9, 11
    x = torch.randn(B, C, T, H, W, generator=g).bfloat16()
    cl = x.permute(0, 2, 3, 4, 1).reshape(B * T * H * W, C)
    ld = C + 8
    xd = torch.zeros(B * T * H * W, ld, dtype=torch.bfloat16)
    xd[:, :C] = cl
    want, _ = _unfold_ref(x.float(), kernel, stride, pad)  # columns (c, taps)
    kv = kernel[0] * kernel[1] * kernel[2]
    want = want.view(-1, C, kv).transpose(1, 2).reshape(-1, kv * C)  # -> (taps, c)
    out = torch.zeros(want.shape[0], kv * C, dtype=torch.bfloat16, device=DEV)
    ops().conv3d_im2col(xd.to(DEV), "cl_bf16", B, (T, H, W), C, kernel, stride, pad, out)
    assert torch.equal(out.cpu(), want.bfloat16())


def test_maxpool3d():
    g = torch.Generator().manual_seed(2)
    B, C, T, H, W = 2, 16, 3, 13, 12
    x = torch.randn(B, C, T, H, W, generator=g).bfloat16()
    want = torch.nn.functional.max_pool3d(x.float(), (1, 3, 3), (1, 2, 2), (0, 1, 1))
    To, Ho, Wo = want.shape[2:]
    out = torch.zeros(B * To * Ho * Wo, C, dtype=torch.bfloat16, device=DEV)
    ops().maxpool3d(x.permute(0, 2, 3, 4, 1).reshape(-1, C).contiguous().to(DEV), B, (T, H, W), C, (1, 3, 3), (1, 2, 2),
                    (0, 1, 1), out)
    assert torch.equal(out.cpu(), want.permute(0, 2, 3, 4, 1).reshape(-1, C).bfloat16())


def test_avgpool_head():
    g = torch.Generator().manual_seed(3)
    B, C, T, H, W = 2, 256, 9, 7, 7
    x = torch.randn(B, C, T, H, W, generator=g).bfloat16().float()
    wc, bc = torch.randn(2, C, generator=g) * 0.05, torch.randn(2, generator=g)
    pooled = torch.nn.functional.avg_pool3d(x, (4, 7, 7), stride=1)
    want = (pooled.permute(0, 2, 3, 4, 1) @ wc.T + bc).mean(dim=(1, 2, 3))
    out = torch.zeros(B, 2, device=DEV)
    ops().avgpool_head(x.permute(0, 2, 3, 4, 1).reshape(-1, C).bfloat16().contiguous().to(DEV), B, (T, H, W), C,
                       (4, 7, 7), wc.to(DEV), bc.to(DEV), torch.zeros(B * C * 33, device=DEV), out)
    assert torch.allclose(out.cpu(), want, atol=1e-4)


def _model():
    from vclip_amd.resnet3d import ResNet3d
    m = ResNet3d(ref.RESNET3D_50)
    m.load_state_dict(make_resnet3d_weights(ref.RESNET3D_50, seed=0))
    return m.to(DEV).eval()


@pytest.mark.parametrize("T,B", [(8, 2), (32, 1)])
def test_resnet3d_logits(T, B):
    video = make_synthetic_video(B, T, 224, seed=2)
    sd = {k: torch.from_numpy(v) for k, v in make_resnet3d_weights(ref.RESNET3D_50, seed=0).items()}
    with torch.no_grad():
        want = ref.resnet3d_forward(sd, ref.RESNET3D_50, torch.from_numpy(video)).numpy()
    got = _model()(torch.from_numpy(video).to(DEV)).cpu().numpy()
    err = np.abs(got - want).max()
    assert err < 1e-2 * max(1.0, np.abs(want).max()), (err, got, want)


def test_resnet3d_batch_invariance():
    video = torch.from_numpy(make_synthetic_video(3, 8, 224, seed=4)).to(DEV)
    m = _model()
    full = m(video).clone()
    one = m(video[1:2].contiguous()).clone()
    assert torch.equal(full[1:2], one)


def test_resnet3d_b4_bench_path_graphed():
    """bench.py --mode resnet3d's timed configuration: B = 4 32x224^2 clips over 2 concurrent HIP streams,
    replayed from the captured hipGraph.  A FRESH model's first call (packing, workspaces, the padding
    row) goes straight into the split + capture; its logits and a second input tensor's (served by the
    static-buffer capture) must equal the one-stream eager forward bit for bit, and the oracle within
    the file's relative bar."""
    video = torch.from_numpy(make_synthetic_video(4, 32, 224, seed=3)).to(DEV)
    video2 = torch.flip(video, dims=[0]).contiguous()
    m = _model()
    m.concurrent_streams = 2
    m.graph_replay = True
    got = m.forward_logits(video).clone()
    got2 = m.forward_logits(video2.clone()).clone()
    again = m.forward_logits(video).clone()
    eager_m = _model()
    want = eager_m.forward_logits(video).clone()
    want2 = eager_m.forward_logits(video2).clone()
    assert torch.equal(got, want) and torch.equal(again, want)
    assert torch.equal(got2, want2)
    sd = {k: torch.from_numpy(v) for k, v in make_resnet3d_weights(ref.RESNET3D_50, seed=0).items()}
    with torch.no_grad():
        r = ref.resnet3d_forward(sd, ref.RESNET3D_50, video[:1].cpu()).numpy()
    err = np.abs(got[:1].cpu().numpy() - r).max()
    assert err < 1e-2 * max(1.0, np.abs(r).max()), (err, got[:1], r)


@pytest.mark.parametrize("kernel,stride,pad,C,epi", [((1, 3, 3), (1, 2, 2), (0, 1, 1), 64, "bias_relu"),
                                                      ((1, 3, 3), (1, 1, 1), (0, 1, 1), 128, "bias_relu"),
                                                      ((3, 1, 1), (1, 1, 1), (1, 0, 0), 64, "bias_relu"),
                                                      ((1, 1, 1), (1, 2, 2), (0, 0, 0), 128, "bias"),
                                                      ((1, 3, 3), (1, 1, 1), (0, 1, 1), 64, "bias_resid_relu"),
                                                      ((1, 3, 3), (1, 2, 2), (0, 1, 1), 64, "bias_relu_n64"),
                                                      ((1, 1, 1), (1, 1, 1), (0, 0, 0), 128, "bias_relu_n64")])
def test_conv3d_implicit_gemm_bit_exact(kernel, stride, pad, C, epi):
    """vc_conv3d_gemm_bf16 (A rows gathered per tap, zero rows for padding taps) == im2col + vc_gemm
    on the same weights: the same MFMA chain per output element, so bit-identical; odd spatial sizes
    put padding taps on every border, and 203 output rows leave a partial 128-row tile."""
    O = ops()
    g = torch.Generator().manual_seed(C + kernel[0])
    B, T, H, W = 2, 4, 13, 11
    N = 128
    n64 = epi.endswith("_n64")  # 64 output channels: the 256 x 64 tile, compared with the first 64 columns
    epi = epi.replace("_n64", "")
    kv = kernel[0] * kernel[1] * kernel[2]
    x = (torch.randn(B * T * H * W, C, generator=g) * 0.5).bfloat16()
    xd = torch.zeros(B * T * H * W, C + 64, dtype=torch.bfloat16)  # ldx > C
    xd[:, :C] = x
    xd = xd.to(DEV)
    w = (torch.randn(N, kv * C, generator=g) * 0.05).bfloat16().to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    To, Ho, Wo = O.conv_out_size((T, H, W), kernel, stride, pad)
    M = B * To * Ho * Wo
    Mp = (M + 255) // 256 * 256
    aux = (torch.randn(Mp, N, generator=g)).bfloat16().to(DEV) if epi == "bias_resid_relu" else None
    col = torch.zeros(Mp, kv * C, dtype=torch.bfloat16, device=DEV)
    O.conv3d_im2col(xd, "cl_bf16", B, (T, H, W), C, kernel, stride, pad, col)
    want = torch.zeros(Mp, N, dtype=torch.bfloat16, device=DEV)
    O.gemm(col, w, b, epi, want, aux=aux, cfg=5)
    got = torch.full((Mp, N), 7.0, dtype=torch.bfloat16, device=DEV)
    O.conv3d_gemm(xd, B, (T, H, W), C, kernel, stride, pad, w, b, epi, got, aux=aux, n=64 if n64 else None, ring=2)
    nc = 64 if n64 else N
    assert torch.equal(got[:M, :nc], want[:M, :nc])
    # the 3-deep LDS ring (vc_conv3d_gemm_bf16_ring; what the automatic choice runs on this small grid):
    # the same MFMA chain, bit-identical
    got3 = torch.full((Mp, N), 7.0, dtype=torch.bfloat16, device=DEV)
    O.conv3d_gemm(xd, B, (T, H, W), C, kernel, stride, pad, w, b, epi, got3, aux=aux, n=64 if n64 else None, ring=3)
    assert torch.equal(got3[:M, :nc], want[:M, :nc])
    # every tile / ring vc_conv3d_gemm_bf16_cfg accepts here (64 x 128 takes bias / bias_relu only; ring 4
    # is one workgroup per CU, 3 on the 256 x 64 tile): bit-identical too
    tiles = (0,) if n64 else ((0, 1, 2) if epi != "bias_resid_relu" else (0, 2))
    for tile in tiles:
        for ring in (0, 2, 3, 4):
            gt = torch.full((Mp, N), 7.0, dtype=torch.bfloat16, device=DEV)
            O.conv3d_gemm(xd, B, (T, H, W), C, kernel, stride, pad, w, b, epi, gt, aux=aux, n=64 if n64 else None,
                          ring=ring, tile=tile)
            assert torch.equal(gt[:M, :nc], want[:M, :nc]), (tile, ring)


def test_resnet3d_split_sizes_and_conv_cfg_bit_identical():
    """Uneven stream parts (model.split_sizes) and per-convolution tile / ring overrides (model.conv_cfg)
    change only the schedule: logits bit-identical to the one-stream default."""
    video = torch.from_numpy(make_synthetic_video(3, 8, 224, seed=9)).to(DEV)
    m = _model()
    ref = m(video).clone()
    m.concurrent_streams, m.split_sizes = 2, [2, 1]
    assert torch.equal(m(video), ref)
    m.concurrent_streams, m.split_sizes = 1, None
    m.conv_cfg = {"conv_a.s4": (4, 1), "conv_b.s4": (2, 2), "conv_b.s3": (3, 2), "conv_a.s5": (3, 1)}
    assert torch.equal(m(video), ref)


def test_resnet3d_implicit_conv_matches_im2col_path():
    """The whole forward with the implicit convolutions (vc_conv3d_gemm_bf16 and the implicit stem)
    vs im2col + GEMM.  The bottleneck convolutions are bit-identical (same column order); the stem sums
    its 441 products in (kt, kh, kw, c) order instead of (c, kt, kh, kw), so the logits agree to bf16
    rounding (1e-2 relative, the family's bar), not bit for bit."""
    video = torch.from_numpy(make_synthetic_video(2, 8, 224, seed=5)).to(DEV)
    m = _model()
    m.implicit_conv = True
    a = m(video).clone()
    m.implicit_conv = False
    b = m(video).clone()
    assert float((a - b).abs().max()) <= 1e-2 * max(1.0, float(b.abs().max())), (a, b)


def test_resnet3d_stem_odd_padded_width_falls_back():
    """The implicit stem reads 16-B aligned 8-pixel rows of the padded clip, so an odd padded width (image
    width 225 -> 231) must take the im2col stem.  The bottleneck convolutions are bit-identical between
    the implicit and the im2col paths, so with the stem on im2col in both the whole forward is too (the
    implicit stem would differ by bf16 rounding); and the stem GEMM entry rejects such a width itself."""
    v = torch.from_numpy(make_synthetic_video(1, 8, 224, seed=6))
    video = torch.cat([v, v[..., -1:]], dim=-1).contiguous().to(DEV)  # W = 225
    m = _model()
    m.implicit_conv = True
    a = m(video).clone()
    m.implicit_conv = False
    b = m(video).clone()
    assert torch.equal(a, b), (a, b)
    O = ops()
    x = torch.randn(1, 3, 4, 20, 19, device=DEV)  # padded width 25
    xp = torch.zeros(1 * 6 * 26 * 25 * 4, dtype=torch.bfloat16, device=DEV)
    O.conv3d_stem_pack(x, (1, 3, 3), xp)
    w = torch.zeros(128, 64 * 11, dtype=torch.bfloat16, device=DEV)
    out = torch.zeros(1024, 128, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="even"):
        O.conv3d_stem_gemm(xp, 1, (4, 20, 19), (3, 7, 7), (1, 2, 2), (1, 3, 3), w, torch.zeros(128, device=DEV),
                           "bias_relu", out)


@pytest.mark.parametrize("T,H,W", [(4, 20, 18), (3, 17, 22)])
def test_conv3d_stem_implicit_gemm_matches_im2col(T, H, W):
    """The implicit stem (vc_conv3d_stem_pack + vc_conv3d_stem_gemm_bf16, one 32-column segment per
    (kt, kh) tap row) == im2col (NCTHW f32) + GEMM on the same BN-folded weights: each output is the
    same products in a different k order, so the comparison is to fp32 of the bf16 operands (both
    accumulate in f32): <= 1e-3 relative, plus bit-identical zero padding behaviour at the borders."""
    O = ops()
    g = torch.Generator().manual_seed(T * 100 + H)
    B, C, N = 2, 3, 128
    kernel, stride, pad = (3, 7, 7), (1, 2, 2), (1, 3, 3)
    x = torch.randn(B, C, T, H, W, generator=g)
    w = torch.randn(64, C, *kernel, generator=g) * 0.05
    b = torch.randn(N, generator=g) * 0.1
    To, Ho, Wo = O.conv_out_size((T, H, W), kernel, stride, pad)
    M = B * To * Ho * Wo
    Mp = (M + 255) // 256 * 256
    # im2col path: columns (c, kt, kh, kw)
    K = C * 3 * 7 * 7
    Kp = (K + 63) // 64 * 64
    col = torch.zeros(Mp, Kp, dtype=torch.bfloat16, device=DEV)
    O.conv3d_im2col(x.to(DEV), "ncthw_f32", B, (T, H, W), C, kernel, stride, pad, col)
    wa = torch.zeros(N, Kp)
    wa[:64, :K] = w.reshape(64, K)
    want = torch.zeros(Mp, N, dtype=torch.bfloat16, device=DEV)
    O.gemm(col, wa.bfloat16().to(DEV), b.to(DEV), "bias_relu", want)
    # implicit path: segment columns
    ws_ = torch.zeros(64, 3, 7, 8, 4)
    ws_[:, :, :, :7, :C] = w.permute(0, 2, 3, 4, 1)
    wsg = torch.zeros(N, 64 * 11)
    wsg[:64, :21 * 32] = ws_.reshape(64, 21 * 32)
    xp = torch.zeros(B * (T + 2) * (H + 6) * (W + 6) * 4, dtype=torch.bfloat16, device=DEV)
    O.conv3d_stem_pack(x.to(DEV), pad, xp)
    got = torch.full((Mp, N), 3.0, dtype=torch.bfloat16, device=DEV)
    O.conv3d_stem_gemm(xp, B, (T, H, W), kernel, stride, pad, wsg.bfloat16().to(DEV), b.to(DEV), "bias_relu", got)
    d = (got[:M].float() - want[:M].float()).abs()
    assert float(d.max()) <= 1e-2 * float(want[:M].float().abs().max()), float(d.max())
    # the packed clip is the zero-padded channels-last bf16 of x
    ref = torch.nn.functional.pad(x, (3, 3, 3, 3, 1, 1)).permute(0, 2, 3, 4, 1)
    ref = torch.cat([ref, torch.zeros(*ref.shape[:-1], 1)], -1).bfloat16()
    assert torch.equal(xp.view(ref.shape).cpu(), ref)


@pytest.mark.parametrize("K,cfg", [(64, 5), (128, 5), (512, 5), (512, 8)])
def test_gemm_bias_resid_relu_epilogue(K, cfg):
    """conv_c's epilogue (relu(A.W^T + bias + residual), bf16 residual prefetched before the k loop in
    the 128x128 kernel) against an fp32 torch reference of the same bf16 operands: <= one bf16 ulp of
    the output plus f32 summation-order noise."""
    O = ops()
    g = torch.Generator().manual_seed(K + cfg)
    M, N = 1024, 256
    a = (torch.randn(M, K, generator=g) * 0.5).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    b = torch.randn(N, generator=g) * 0.1
    r = torch.randn(M, N, generator=g).bfloat16()
    want = torch.relu(a.float() @ w.float().T + b + r.float())
    out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    O.gemm(a.to(DEV), w.to(DEV), b.to(DEV), "bias_resid_relu", out, aux=r.to(DEV), cfg=cfg)
    got = out.float().cpu()
    assert torch.allclose(got, want, rtol=2 ** -7, atol=1e-3), float((got - want).abs().max())


@pytest.mark.parametrize("M,N,K,lda,ldr", [(1024, 256, 64, 64, 256), (8192, 512, 128, 256, 512),
                                           (401408, 256, 64, 64, 256), (100352, 512, 128, 128, 512),
                                           (25600, 768, 64, 192, 1024), (2048, 384, 256, 256, 384),
                                           (25088, 1024, 256, 512, 1024)])
def test_conv_c_stream_bit_identical(M, N, K, lda, ldr):
    """The streaming conv_c kernel (cfg 20: W tile resident in LDS, the next m tile's A rows and
    residual in flight under the current tile) against the 128x128 kernel (cfg 5): same MFMA chain and
    epilogue order per output -> bit-identical; strided A (a column slice of a wider buffer, as
    resnet3d passes act["b"][:, :inner]), padded residual rows, fewer m tiles than workgroups and the
    res2 / res3 full sizes."""
    O = ops()
    g = torch.Generator(device=DEV).manual_seed(M + K)
    abuf = (torch.randn(M, lda, device=DEV, generator=g) * 0.5).bfloat16()
    a = abuf[:, :K]
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    rbuf = torch.randn(M, ldr, device=DEV, generator=g).bfloat16()
    r = rbuf[:, :N]
    want = torch.full((M, N), 7.0, dtype=torch.bfloat16, device=DEV)
    assert O.gemm_kernel_name(M, N, K, "bias_resid_relu", want, r, cfg=20).startswith(f"conv_c_stream_kernel<{K}, ")
    if K <= 128 and N % 256 == 0:  # the default pick for conv_c at K 64 / 128
        assert O.gemm_kernel_name(M, N, K, "bias_resid_relu", want, r) == f"conv_c_stream_kernel<{K}, 256>"
    got = want.clone()
    O.gemm(a, w, b, "bias_resid_relu", want, aux=r, cfg=5)
    O.gemm(a, w, b, "bias_resid_relu", got, aux=r, cfg=20)
    torch.cuda.synchronize()
    assert torch.equal(got, want), int((got != want).sum())
    if M <= 8192:  # and the fp32 torch reference
        ref = torch.relu(a.float() @ w.float().T + b + r.float())
        assert torch.allclose(got.float(), ref, rtol=2 ** -7, atol=1e-3)


def test_conv_c_stream_alignment_gate():
    """cfg 20 moves 16-B pieces of out and of the bf16 residual: with a residual row stride that is not a
    multiple of 8 elements the automatic pick falls back to cfg 5 (same result) and an explicit cfg 20
    is rejected instead of running misaligned 16-B accesses."""
    O = ops()
    M, N, K = 1024, 256, 64
    g = torch.Generator(device=DEV).manual_seed(5)
    a = (torch.randn(M, K, device=DEV, generator=g) * 0.5).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    rbuf = torch.randn(M, N + 4, device=DEV, generator=g).bfloat16()
    r = rbuf[:, :N]  # ldaux = N + 4: 8-B aligned rows, not 16-B
    assert O.gemm_kernel_name(M, N, K, "bias_resid_relu", torch.empty(M, N, device=DEV), r).startswith(
        "gemm_bf16_kernel<128, 128")
    want = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    got = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    O.gemm(a, w, b, "bias_resid_relu", want, aux=r, cfg=5)
    O.gemm(a, w, b, "bias_resid_relu", got, aux=r)
    assert torch.equal(got, want)
    with pytest.raises(RuntimeError, match="cfg 20"):
        O.gemm(a, w, b, "bias_resid_relu", got, aux=r, cfg=20)
