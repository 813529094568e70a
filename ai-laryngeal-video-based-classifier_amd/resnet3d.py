"""3D ResNet-50 (pytorchvideo `create_resnet` as the reference configures it) on the
libvclip.so kernels — drop-in for `create_model(logger)` of
resnet50-3d-video/video_classifier/models/resnet3d.py:4-48, called as
`model(f32[B, 3, T, H, W])` -> `f32[B, 2]` (resnet50-3d-video trainer / inference.py:399).

Every Conv3d + BatchNorm(eval) [+ ReLU] [+ residual] is one GEMM: BN is folded into the
weights and bias in fp32 before the bf16 cast, ReLU and the bottleneck's skip add are GEMM
epilogues; 1x1x1 stride-1 convolutions read the activations directly, the others go through
vc_conv3d_im2col.  Activations are channels-last bf16 rows ((b*T + t)*H + h)*W + w; rows are
padded to a multiple of 256 and output channels to a multiple of 128 (zero weights, so the
padding columns are exactly 0).  The head (AvgPool3d (4,7,7) stride 1 -> Linear ->
global average) is one position-weighted pooling + GEMV (the Linear commutes with both means).

Parity unpinned against pytorchvideo itself (not installed here): checked against
oracle/resnet3d_ref.py, the restatement of pytorchvideo's create_resnet.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from . import ops, streams
from .weights import resnet3d_param_shapes

RESNET3D_50 = dict(depths=(3, 4, 6, 3), stem_dim=64, conv_a_kernels=((1, 1, 1), (1, 1, 1), (3, 1, 1), (3, 1, 1)),
                   spatial_strides=(1, 2, 2, 2), head_pool=(4, 7, 7), num_classes=2, bn_eps=1e-5,
                   stem_kernel=(3, 7, 7), stem_pad=(1, 3, 3))


def _ru(x, m):
    return (x + m - 1) // m * m


class ResNet3d(torch.nn.Module):
    """fp32 master parameters + BatchNorm running statistics in pytorchvideo naming."""

    def __init__(self, cfg: dict = RESNET3D_50):
        super().__init__()
        self.cfg = dict(cfg)
        shapes = resnet3d_param_shapes(self.cfg)
        self._names = list(shapes.keys())
        self.params = torch.nn.ParameterDict()
        for n, s in shapes.items():
            # BatchNorm running statistics are buffers in pytorchvideo: no gradient, updated by the train step
            stat = n.endswith("running_mean") or n.endswith("running_var")
            self.params[n.replace(".", "__")] = torch.nn.Parameter(torch.zeros(s), requires_grad=not stat)
        self._packed = None
        self._ws = {}
        self._ws_used = []
        self.concurrent_streams = None  # n > 1: the inference batch split over n HIP streams (vclip_amd.streams)
        self.split_sizes = None  # clips per stream part (streams.run_split); None = as even as possible
        self._streams = None
        self._split_out = {}
        # True: the inference forward is captured once per input / configuration into a hipGraph and
        # replayed (streams.GraphReplay); bit-identical logits
        self.graph_replay = False
        self._graphs = None
        self.head_dropout = True  # train step: the head's Dropout(0.5) (pytorchvideo create_resnet dropout_rate)
        # inference convolutions other than 1x1x1 stride 1 as implicit GEMMs (vc_conv3d_gemm_bf16: the
        # A rows gathered from the activations per kernel tap, no im2col buffer); False: im2col + GEMM.
        # The bottleneck convolutions are bit-identical either way (same MFMA chain per output, same
        # column order); the implicit stem sums its 441 products in another k order, so the stem (and
        # the logits) agree with the im2col path to bf16 rounding.
        self.implicit_conv = True
        # LDS ring depth of the implicit convolutions per res stage ("s2" .. "s5" -> 2 or 3;
        # vc_conv3d_gemm_bf16_ring), absent = automatic by grid size (bit-identical for any setting)
        self.conv_ring = {}
        # per-convolution overrides {"conv_a.s4": (ring, tile), ...} of vc_conv3d_gemm_bf16_cfg (tile 0 auto,
        # 1 = 64 x 128, 2 = 128 x 128; ring 0 auto, 2, 3, 4); bit-identical for any setting
        self.conv_cfg = {}

    def _conv_kw(self, op: str, s: int) -> dict:
        ring, tile = self.conv_cfg.get(op, (self.conv_ring.get(f"s{s + 2}", 0), 0))
        return dict(ring=ring, tile=tile)

    def state_dict(self, *a, **k):
        return OrderedDict((n, self.params[n.replace(".", "__")].detach()) for n in self._names)

    def load_state_dict(self, sd, strict: bool = True):
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
        sd = {k: v for k, v in sd.items() if not k.endswith("num_batches_tracked")}
        missing = [n for n in self._names if n not in sd]
        unexpected = [k for k in sd if k not in self._names]
        if strict and (missing or unexpected):
            raise KeyError(f"load_state_dict: missing={missing[:5]} unexpected={unexpected[:5]}")
        with torch.no_grad():
            for n in self._names:
                if n in sd:
                    v = sd[n]
                    v = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
                    dst = self.params[n.replace(".", "__")]
                    dst.copy_(v.reshape(dst.shape))
        self._packed = None
        return missing, unexpected

    # ---- packing: BN folded, weights [N_pad, K] bf16 in the im2col column order --------
    def P(self, name):
        return self.params[name.replace(".", "__")]

    def _weights_version(self):
        from . import vivit_train
        return (vivit_train.MASTER_EPOCH[0], sum(p._version for p in self.params.values()))

    def _pack(self, device):
        ver = self._weights_version()  # the fused AdamW updates in place without bumping _version
        if self._packed is not None and self._packed["device"] == device and self._packed["version"] == ver:
            return self._packed
        ops.zero_row(device)  # the implicit convs' padding row, zeroed on the caller's stream before any fork
        c = self.cfg
        eps = c["bn_eps"]
        P = lambda n: self.params[n.replace(".", "__")].detach().to(device=device, dtype=torch.float64)  # noqa: E731

        def fold(conv, bn, channels_last=True, k_pad=None):
            w = P(conv + ".weight")
            sc = P(bn + ".weight") / torch.sqrt(P(bn + ".running_var") + eps)
            b = P(bn + ".bias") - P(bn + ".running_mean") * sc
            w = w * sc.view(-1, 1, 1, 1, 1)
            w = (w.permute(0, 2, 3, 4, 1) if channels_last else w).reshape(w.shape[0], -1)
            n_p = _ru(w.shape[0], 128)
            k = w.shape[1] if k_pad is None else k_pad
            W = torch.zeros((n_p, k), dtype=torch.float64, device=device)
            W[:w.shape[0], :w.shape[1]] = w
            B = torch.zeros(n_p, dtype=torch.float64, device=device)
            B[:b.numel()] = b
            return W.to(torch.bfloat16).contiguous(), B.float().contiguous()

        pk = {"device": device, "version": ver}
        sk = c.get("stem_kernel", (3, 7, 7))
        pk["stem"] = fold("blocks.0.conv", "blocks.0.norm", channels_last=False, k_pad=_ru(3 * sk[0] * sk[1] * sk[2], 64))
        if sk[2] <= 8:
            # the implicit stem GEMM's segment columns: seg = kt_i * kh + kh_i, column seg*32 + kw_i*4 + c
            w = P("blocks.0.conv.weight")
            scl = P("blocks.0.norm.weight") / torch.sqrt(P("blocks.0.norm.running_var") + eps)
            w = w * scl.view(-1, 1, 1, 1, 1)
            co, ci = w.shape[0], w.shape[1]
            nseg = sk[0] * sk[1]
            Wseg = torch.zeros((_ru(co, 128), 64 * ((nseg + 1) // 2)), dtype=torch.float64, device=device)
            ws_ = torch.zeros((co, sk[0], sk[1], 8, 4), dtype=torch.float64, device=device)
            ws_[:, :, :, :sk[2], :ci] = w.permute(0, 2, 3, 4, 1)
            Wseg[:co, :nseg * 32] = ws_.reshape(co, nseg * 32)
            pk["stem_seg"] = (Wseg.to(torch.bfloat16).contiguous(), pk["stem"][1])
        stages = []
        din, dout = c["stem_dim"], c["stem_dim"] * 4
        for s, depth in enumerate(c["depths"]):
            blocks = []
            for i in range(depth):
                p = f"blocks.{s + 1}.res_blocks.{i}."
                blk = {}
                if p + "branch1_conv.weight" in self._names:
                    blk["b1"] = fold(p + "branch1_conv", p + "branch1_norm")
                blk["a"] = fold(p + "branch2.conv_a", p + "branch2.norm_a")
                blk["b"] = fold(p + "branch2.conv_b", p + "branch2.norm_b")
                blk["c"] = fold(p + "branch2.conv_c", p + "branch2.norm_c")
                blocks.append(blk)
            stages.append(dict(blocks=blocks, din=din, dout=dout, inner=dout // 4))
            din, dout = dout, dout * 2
        pk["stages"] = stages
        if "blocks.5.proj.weight" in self._names:
            pk["w_head"] = self.params["blocks__5__proj__weight"].detach().to(device).float().contiguous()
            pk["b_head"] = self.params["blocks__5__proj__bias"].detach().to(device).float().contiguous()
        self._packed = pk
        return pk

    # ---- geometry / workspace ---------------------------------------------------------
    def geometry(self, T, H, W):
        c = self.cfg
        stem = ops.conv_out_size((T, H, W), c.get("stem_kernel", (3, 7, 7)), (1, 2, 2), c.get("stem_pad", (1, 3, 3)))
        g = [ops.conv_out_size(stem, (1, 3, 3), (1, 2, 2), (0, 1, 1))]
        for s in range(1, len(c["depths"])):
            st = c["spatial_strides"][s]
            g.append(ops.conv_out_size(g[-1], (1, 3, 3), (1, st, st), (0, 1, 1)))
        return stem, g

    def _workspace(self, B, T, H, W, device, part: int = 0):
        key = (B, T, H, W, str(device), part)
        if key in self._ws:
            ws = self._ws[key]
            if not any(w is ws for w in self._ws_used):
                self._ws_used.append(ws)
            return ws
        if len(self._ws) >= 4:
            self._ws = {}
        c = self.cfg
        stem, grids = self.geometry(T, H, W)
        bf = torch.bfloat16
        rows = lambda g: _ru(B * g[0] * g[1] * g[2], 256)  # noqa: E731
        z = lambda r, cols: torch.zeros((r, cols), dtype=bf, device=device)  # noqa: E731
        ws = {"stem_out": z(rows(stem), 128)}
        sp = c.get("stem_pad", (1, 3, 3))
        # + 8 pixels x 4 channels of slack: the implicit stem reads 8 pixels per tap row, so with kw < 8 the
        # last output window of the last row reads up to 8 - kw pixels past the packed clip (zero weights)
        ws["stem_pad"] = torch.zeros(B * (T + 2 * sp[0]) * (H + 2 * sp[1]) * (W + 2 * sp[2]) * 4 + 32, dtype=bf,
                                     device=device)
        # im2col scratch: the largest M x K of any convolution
        sk = c.get("stem_kernel", (3, 7, 7))
        big = rows(stem) * _ru(3 * sk[0] * sk[1] * sk[2], 64)
        din, dout = c["stem_dim"], c["stem_dim"] * 4
        g_in = grids[0]
        acts = []
        for s, depth in enumerate(c["depths"]):
            g = grids[s]
            inner = dout // 4
            ka = c["conv_a_kernels"][s]
            big = max(big, rows(g_in) * ka[0] * ka[1] * ka[2] * max(din, dout), rows(g) * 9 * inner,
                      rows(g) * din)
            acts.append(dict(x=z(rows(g), dout), x2=z(rows(g), dout), sc=z(rows(g), dout),
                             a=z(rows(g_in) if g_in != g else rows(g), _ru(inner, 128)), b=z(rows(g), _ru(inner, 128))))
            g_in = g
            din, dout = dout, dout * 2
        ws["x0"] = z(rows(grids[0]), c["stem_dim"])
        ws["acts"] = acts
        # im2col scratch (1.4 GB at B = 4 for the stem alone): allocated on first use, i.e. only by the
        # im2col path (implicit_conv = False)
        ws["col"] = None
        ws["col_elems"] = big
        ws["head_work"] = torch.zeros(B * T * 2048 * 33, dtype=torch.float32, device=device)
        ws["logits"] = torch.zeros((B, c["num_classes"]), dtype=torch.float32, device=device)
        self._ws[key] = ws
        self._ws_used.append(ws)
        return ws

    # ---- forward -----------------------------------------------------------------------
    def forward(self, video: torch.Tensor) -> torch.Tensor:
        """`model(clips)` -> logits.  In training mode (the reference's train loop,
        resnet50-3d-video/video_classifier/trainers/trainer.py:106-123) the HIP train step runs
        (_forward_train: BatchNorm with batch statistics and running-statistic updates, the head's
        dropout), with autograd enabled or not -- pytorchvideo in train mode under torch.no_grad keeps
        those semantics too; in eval mode the fused inference path (BatchNorm folded) runs."""
        if video.device.type != "cuda":
            raise RuntimeError("ResNet3d (vclip_amd) runs on the GPU only: move the clip batch to cuda")
        x = video.contiguous().float() if video.dtype != torch.float32 else video.contiguous()
        if self.training:
            return self._forward_train(x)
        with torch.no_grad():
            return self.forward_logits(x).clone()  # the workspace buffer is reused by the next call

    def _forward_train(self, video: torch.Tensor) -> torch.Tensor:
        """pytorchvideo create_resnet in training mode (oracle/resnet3d_ref.py with batch-statistic
        BatchNorm) as autograd ops over the HIP kernels (vclip_amd/autograd_ops.py): every Conv3d is
        an im2col (differentiable: col2im) + bf16 MFMA GEMM with fp32 accumulation on the fp32 master
        weights, BatchNorm3d with batch statistics (fp32, running statistics updated with momentum
        0.1) fused with the residual add and ReLU, MaxPool3d with its first-max gradient, and the head
        (AvgPool3d, Dropout(0.5) from torch's RNG unless `head_dropout = False`, Linear, global
        average); channels-last rows throughout."""
        from . import autograd_ops as A
        c = self.cfg
        B, Cin, T, H, W = video.shape
        if Cin != 3:
            raise ValueError("video must be [B, 3, T, H, W]")
        eps = c["bn_eps"]
        stem, grids = self.geometry(T, H, W)
        sk, sp = c.get("stem_kernel", (3, 7, 7)), c.get("stem_pad", (1, 3, 3))
        P = self.P

        def bn(y, name, relu, res=None):
            return A.batchnorm(y, P(name + ".weight"), P(name + ".bias"), P(name + ".running_mean"),
                               P(name + ".running_var"), res=res, relu=relu, eps=eps)

        def conv(x, grid, cin, wname, kernel, stride, pad):
            w = P(wname)
            cout = w.shape[0]
            if tuple(kernel) == (1, 1, 1) and tuple(stride) == (1, 1, 1):
                a = x
            else:
                a = A.im2col_cl(x, B, grid, cin, kernel, stride, pad)
            return A.linear(a, w.permute(0, 2, 3, 4, 1).reshape(cout, -1), None, out_f32=True)

        # stem: Conv3d from the f32 NCTHW clip (no input gradient) + BN + ReLU + MaxPool
        Ms = B * stem[0] * stem[1] * stem[2]
        K = 3 * sk[0] * sk[1] * sk[2]
        a = torch.empty(Ms, _ru(K, 8), dtype=torch.bfloat16, device=video.device)
        ops.conv3d_im2col(video, "ncthw_f32", B, (T, H, W), 3, sk, (1, 2, 2), sp, a)
        y = A.linear(a[:, :K], P("blocks.0.conv.weight").reshape(c["stem_dim"], K), None, out_f32=True)
        x = A.maxpool(bn(y, "blocks.0.norm", True), B, stem, c["stem_dim"], (1, 3, 3), (1, 2, 2), (0, 1, 1))
        g_in, cin = grids[0], c["stem_dim"]
        for s, depth in enumerate(c["depths"]):
            g = grids[s]
            ss = c["spatial_strides"][s]
            ka = tuple(c["conv_a_kernels"][s])
            for i in range(depth):
                p = f"blocks.{s + 1}.res_blocks.{i}."
                stride = (1, ss, ss) if i == 0 else (1, 1, 1)
                gi = g_in if i == 0 else g
                if p + "branch1_conv.weight" in self._names:
                    sc = bn(conv(x, gi, cin, p + "branch1_conv.weight", (1, 1, 1), stride, (0, 0, 0)),
                            p + "branch1_norm", False)
                else:
                    sc = x
                inner = P(p + "branch2.conv_a.weight").shape[0]
                ya = bn(conv(x, gi, cin, p + "branch2.conv_a.weight", ka, (1, 1, 1), tuple(k // 2 for k in ka)),
                        p + "branch2.norm_a", True)
                yb = bn(conv(ya, gi, inner, p + "branch2.conv_b.weight", (1, 3, 3), stride, (0, 1, 1)),
                        p + "branch2.norm_b", True)
                x = bn(conv(yb, g, inner, p + "branch2.conv_c.weight", (1, 1, 1), (1, 1, 1), (0, 0, 0)),
                       p + "branch2.norm_c", True, res=sc)
                cin = P(p + "branch2.conv_c.weight").shape[0]
            g_in = g
        Tf, Hf, Wf = grids[-1]
        pt, ph, pw = c["head_pool"]
        if (ph, pw) != (Hf, Wf):
            raise NotImplementedError("train step head: the pool window must cover the final spatial map")
        npos = Tf - pt + 1
        keep = torch.ones(B, npos, cin, device=video.device)
        if self.head_dropout:
            keep = keep.bernoulli_(0.5).mul_(2.0)  # nn.Dropout(0.5): keep with prob 0.5, scale 1 / 0.5
        self._packed = None  # the running statistics were updated in place: re-fold before the next eval
        return A.resnet_head(x, P("blocks.5.proj.weight"), P("blocks.5.proj.bias"), keep, B, Tf, Hf * Wf, pt)

    def forward_logits(self, video: torch.Tensor) -> torch.Tensor:
        """logits f32 [B, classes] (a workspace buffer, overwritten by the next call); with
        `concurrent_streams = n > 1` the batch is split over n HIP streams (vclip_amd.streams) and with
        `graph_replay` the forward is replayed from a captured hipGraph (bit-identical either way)."""
        if video.shape[1] != 3:
            raise ValueError("video must be [B, 3, T, H, W]")
        if self.graph_replay and not streams.serial() and not torch.cuda.is_current_stream_capturing():
            from .streams import GraphReplay
            if self._graphs is None:
                self._graphs = GraphReplay()
            key = (video.data_ptr(), tuple(video.shape), tuple(video.stride()), video.dtype, self.concurrent_streams, None if self.split_sizes is None else tuple(self.split_sizes),
                   self.implicit_conv, tuple(sorted(self.conv_ring.items())), tuple(sorted(self.conv_cfg.items())),
                   str(video.device), self._weights_version())
            return self._graphs.run(key, video, self._forward_eager, keep=lambda: (self._packed, tuple(self._ws_used)))
        return self._forward_eager(video)

    def _forward_eager(self, video: torch.Tensor) -> torch.Tensor:
        self._ws_used = []  # the workspaces this forward addresses (a captured graph keeps exactly these)
        B = video.shape[0]
        ns = max(1, min(int(self.concurrent_streams or 1), B))
        if ns == 1:
            return self._forward_part(video, 0)
        from .streams import run_split
        return run_split(self, video, ns, self._forward_part, self.cfg["num_classes"],
                         prepare=lambda: self._pack(video.device))

    def _forward_part(self, video: torch.Tensor, part: int, out=None) -> torch.Tensor:
        x, B, grid, C, ws = self.forward_features(video, part)
        pk = self._packed
        c = self.cfg
        Tf, Hf, Wf = grid
        pt, ph, pw = c["head_pool"]
        npos = (Tf - pt + 1) * (Hf - ph + 1) * (Wf - pw + 1)
        return ops.timed("avgpool_head", "head", B * Tf * Hf * Wf * C * 2 + npos * B * C * 4, "byte", ops.avgpool_head,
                         x, B, grid, C, c["head_pool"], pk["w_head"], pk["b_head"], ws["head_work"],
                         ws["logits"] if out is None else out)

    def forward_features(self, video: torch.Tensor, part: int = 0):
        """Stem + the four stages; returns (last activations [rows, C] bf16, B, (T, H, W), C, workspace)."""
        c = self.cfg
        B, C, T, H, W = video.shape
        if C != 3:
            raise ValueError("video must be [B, 3, T, H, W]")
        pk = self._pack(video.device)
        ws = self._workspace(B, T, H, W, video.device, part)
        stem, grids = self.geometry(T, H, W)
        rows = lambda g: _ru(B * g[0] * g[1] * g[2], 256)  # noqa: E731

        def col(m, k):
            if ws["col"] is None:
                ws["col"] = torch.zeros(ws["col_elems"], dtype=torch.bfloat16, device=video.device)
            return ws["col"][: m * k].view(m, k)

        # stem: conv (3,7,7)/(1,2,2) + BN + ReLU, then MaxPool (1,3,3)/(1,2,2)
        # (algorithmic work per launch for an installed ops.OpRecorder: real rows and channels; the
        # GEMMs run on rows padded to 256 and output channels padded to 128)
        tm = ops.timed
        vol = lambda g: B * g[0] * g[1] * g[2]  # noqa: E731
        sk = c.get("stem_kernel", (3, 7, 7))
        ks = 3 * sk[0] * sk[1] * sk[2]
        spad = c.get("stem_pad", (1, 3, 3))
        # (the implicit stem reads 16-B aligned 8-pixel rows of the padded clip: its padded width must be even)
        if self.implicit_conv and "stem_seg" in pk and (W + 2 * spad[2]) % 2 == 0:
            # the clip as zero-padded channels-last bf16 (4 channels), then the implicit stem GEMM
            tm("stem_pack_kernel", "stem_pack", B * 3 * T * H * W * 4 + ws["stem_pad"].numel() * 2, "byte",
               ops.conv3d_stem_pack, video, spad, ws["stem_pad"])
            ops.conv3d_stem_gemm(ws["stem_pad"], B, (T, H, W), sk, (1, 2, 2), spad, pk["stem_seg"][0], pk["stem_seg"][1],
                                 "bias_relu", ws["stem_out"], flop=2.0 * vol(stem) * c["stem_dim"] * ks, op="stem",
                                 n=_ru(c["stem_dim"], 64))
        else:
            Kst = pk["stem"][0].shape[1]
            A = col(rows(stem), Kst)
            tm("conv3d_im2col_kernel", "im2col", B * 3 * T * H * W * 4 + vol(stem) * ks * 2, "byte", ops.conv3d_im2col,
               video, "ncthw_f32", B, (T, H, W), 3, sk, (1, 2, 2), spad, A)
            ops.gemm(A, pk["stem"][0], pk["stem"][1], "bias_relu", ws["stem_out"],
                     flop=2.0 * vol(stem) * c["stem_dim"] * ks, op="stem")
        x = ws["x0"]
        tm("maxpool3d_kernel", "maxpool", (vol(stem) + vol(grids[0])) * c["stem_dim"] * 2, "byte", ops.maxpool3d,
           ws["stem_out"], B, stem, c["stem_dim"], (1, 3, 3), (1, 2, 2), (0, 1, 1), x)
        g_in, cin = grids[0], c["stem_dim"]
        for s, (st, act) in enumerate(zip(pk["stages"], ws["acts"])):
            g = grids[s]
            ss = c["spatial_strides"][s]
            ka = c["conv_a_kernels"][s]
            inner, dout = st["inner"], st["dout"]
            for i, blk in enumerate(st["blocks"]):
                stride = (1, ss, ss) if i == 0 else (1, 1, 1)
                gi = g_in if i == 0 else g
                xin = x
                # branch1: 1x1x1 conv (+ stride) + BN, or the identity
                if "b1" in blk:
                    fl = 2.0 * vol(g) * dout * cin
                    if stride == (1, 1, 1):
                        ops.gemm(xin, blk["b1"][0], blk["b1"][1], "bias", act["sc"], m=rows(g), flop=fl, op=f"branch1.s{s + 2}")
                    elif self.implicit_conv and cin % 64 == 0:
                        ops.conv3d_gemm(xin, B, gi, cin, (1, 1, 1), stride, (0, 0, 0), blk["b1"][0], blk["b1"][1], "bias",
                                        act["sc"], flop=fl, op=f"branch1.s{s + 2}", **self._conv_kw(f"branch1.s{s + 2}", s))
                    else:
                        A = col(rows(g), cin)
                        tm("conv3d_im2col_kernel", "im2col", (vol(gi) + vol(g)) * cin * 2, "byte", ops.conv3d_im2col,
                           xin, "cl_bf16", B, gi, cin, (1, 1, 1), stride, (0, 0, 0), A)
                        ops.gemm(A, blk["b1"][0], blk["b1"][1], "bias", act["sc"], flop=fl, op=f"branch1.s{s + 2}")
                    skip = act["sc"]
                else:
                    skip = xin
                # conv_a (+ BN + ReLU) at the block's input resolution
                fl = 2.0 * vol(gi) * inner * cin * ka[0] * ka[1] * ka[2]
                if tuple(ka) == (1, 1, 1) and self.implicit_conv and inner % 128 and inner % 64 == 0 and cin % 64 == 0:
                    # 64 output channels: the 256 x 64 implicit-GEMM tile (no MFMAs on the zero-padded channels)
                    ops.conv3d_gemm(xin, B, gi, cin, ka, (1, 1, 1), (0, 0, 0), blk["a"][0], blk["a"][1], "bias_relu",
                                    act["a"], flop=fl, op=f"conv_a.s{s + 2}", n=inner, **self._conv_kw(f"conv_a.s{s + 2}", s))
                elif tuple(ka) == (1, 1, 1):
                    ops.gemm(xin, blk["a"][0], blk["a"][1], "bias_relu", act["a"], m=rows(gi), flop=fl, op=f"conv_a.s{s + 2}")
                elif self.implicit_conv and cin % 64 == 0:
                    ops.conv3d_gemm(xin, B, gi, cin, ka, (1, 1, 1), tuple(k // 2 for k in ka), blk["a"][0], blk["a"][1],
                                    "bias_relu", act["a"], flop=fl, op=f"conv_a.s{s + 2}", n=_ru(inner, 64),
                                    **self._conv_kw(f"conv_a.s{s + 2}", s))
                else:
                    A = col(rows(gi), ka[0] * cin)
                    tm("conv3d_im2col_kernel", "im2col", vol(gi) * cin * 2 * (1 + ka[0]), "byte", ops.conv3d_im2col,
                       xin, "cl_bf16", B, gi, cin, ka, (1, 1, 1), tuple(k // 2 for k in ka), A)
                    ops.gemm(A, blk["a"][0], blk["a"][1], "bias_relu", act["a"], flop=fl, op=f"conv_a.s{s + 2}")
                # conv_b (1,3,3) with the stage stride (+ BN + ReLU)
                if self.implicit_conv and inner % 64 == 0:
                    ops.conv3d_gemm(act["a"], B, gi, inner, (1, 3, 3), stride, (0, 1, 1), blk["b"][0], blk["b"][1],
                                    "bias_relu", act["b"], flop=2.0 * vol(g) * inner * inner * 9, op=f"conv_b.s{s + 2}",
                                    n=_ru(inner, 64), **self._conv_kw(f"conv_b.s{s + 2}", s))
                else:
                    A = col(rows(g), 9 * inner)
                    tm("conv3d_im2col_kernel", "im2col", (vol(gi) + 9 * vol(g)) * inner * 2, "byte", ops.conv3d_im2col,
                       act["a"], "cl_bf16", B, gi, inner, (1, 3, 3), stride, (0, 1, 1), A)
                    ops.gemm(A, blk["b"][0], blk["b"][1], "bias_relu", act["b"], flop=2.0 * vol(g) * inner * inner * 9,
                             op=f"conv_b.s{s + 2}")
                # conv_c 1x1x1 + BN + skip + ReLU
                out = act["x"] if xin is not act["x"] else act["x2"]
                # HBM-bound at every stage (K = inner = 64 .. 512 against a bf16 residual in and a bf16
                # output: 28 .. 229 flop/B, below the 312 flop/B ridge): filed under its bytes
                ops.gemm(act["b"][:, :inner], blk["c"][0], blk["c"][1], "bias_resid_relu", out, aux=skip,
                         op=f"conv_c.s{s + 2}", nbytes=2.0 * (vol(g) * (inner + 2 * dout) + dout * inner))
                x, cin = out, dout
            g_in = g
        return x, B, grids[-1], cin, ws


def create_model(logger=None, device="cuda", weights_seed: int = 0):
    """Drop-in for resnet50-3d-video/video_classifier/models/resnet3d.py:4-48 (random init there
    too: `create_resnet` without pretrained weights; here seeded synthetic weights)."""
    if logger:
        logger.info("Creating 3D ResNet-50 model...")
    model = ResNet3d(RESNET3D_50)
    from .weights import make_resnet3d_weights
    model.load_state_dict(make_resnet3d_weights(RESNET3D_50, seed=weights_seed))
    if logger:
        logger.info("Model created successfully")
    return model.to(device) if device else model
