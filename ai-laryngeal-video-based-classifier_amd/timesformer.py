"""TimeSformer-B (divided space-time attention) video classifier on the libvclip.so
kernels — drop-in for the reference's `create_model`
(timesformer/timesformer_classifier/models/timesformer_model.py:4-53), which returns an
HF `TimesformerForVideoClassification` called as `model(pixel_values=...)` and read
through `.logits` (timesformer/timesformer_classifier/trainers/trainer.py, inference.py).

Device data layout (B clips, T frames, P = (image/16)^2 patches, S = 1 + P*T tokens):
  clip layout   rows b*S + r, r = 0 (CLS) or 1 + p*T + t (patch-major, time-minor, the HF
                residual-stream order, TF5/models/timesformer/modeling_timesformer.py:121-143)
  frame layout  rows (b*T + t)*(1 + P) + j, j = 0 (CLS copy) or 1 + p: one spatial
                sequence per frame (:355-364), fed to the joint flash kernel with
                B' = B*T, S' = 1 + P
  both padded to Mpad = roundup(max(B*S, B*T*(1+P)) + 128, 256) rows;
  residual X f32 [Mpad, D] (clip), LN outputs bf16 (clip / frame), q|k|v bf16 [Mpad, 3D],
  attention out bf16 [Mpad, D], branch GEMM out bf16 [Mpad, D], MLP hidden bf16 [Mpad, 4D].
Per layer (TF5/.../modeling_timesformer.py:332-398):
  LN_t -> qkv_t GEMM -> temporal attention (VALU, T keys) -> one GEMM for
  temporal_attention.output.dense followed by temporal_dense (folded: W = Wtd.Wto,
  b = Wtd.bto + btd, in fp32 before the bf16 cast) -> [x += ., LN_before, permute to
  frame layout, CLS copied per frame] -> qkv_s GEMM -> flash attention -> output.dense
  GEMM -> [x += ., CLS += frame mean, LN_after] -> fc1 + exact GELU -> fc2 + residual.
"""
from __future__ import annotations

import json
import math
from collections import OrderedDict

import numpy as np
import torch

from . import ops, streams
from .vivit import ClassifierOutput, _round_up
from .weights import timesformer_param_shapes


class TimesformerConfig:
    """Minimal stand-in for transformers.TimesformerConfig (the fields the path and the
    reference's checkpoint dict use; the factory sets num_classes / video_size too,
    timesformer_model.py:27-31)."""

    defaults = dict(image_size=224, patch_size=16, num_channels=3, num_frames=8, hidden_size=768,
                    num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072, hidden_act="gelu",
                    hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, initializer_range=0.02,
                    layer_norm_eps=1e-6, qkv_bias=True, attention_type="divided_space_time", drop_path_rate=0.0,
                    model_type="timesformer")

    def __init__(self, **kw):
        d = dict(self.defaults)
        d.update(kw)
        id2label = d.pop("id2label", None) or {0: "LABEL_0", 1: "LABEL_1"}
        self.id2label = {int(k): v for k, v in id2label.items()}
        self.label2id = d.pop("label2id", None) or {v: k for k, v in self.id2label.items()}
        d.pop("num_labels", None)
        self.num_classes = d.pop("num_classes", len(self.id2label))
        self.video_size = d.pop("video_size", [d["num_frames"], d["image_size"], d["image_size"]])
        for k, v in d.items():
            setattr(self, k, v)

    @property
    def num_labels(self):
        return len(self.id2label)

    def to_dict(self):
        d = {k: getattr(self, k) for k in self.defaults}
        d["id2label"] = {str(k): v for k, v in self.id2label.items()}
        d["label2id"] = dict(self.label2id)
        d["num_classes"] = self.num_classes
        d["video_size"] = list(self.video_size)
        return d

    @classmethod
    def from_dict(cls, d):
        return cls(**d)

    def as_shape_cfg(self):
        return dict(hidden_size=self.hidden_size, intermediate_size=self.intermediate_size, patch_size=self.patch_size,
                    num_channels=self.num_channels, num_frames=self.num_frames, image_size=self.image_size,
                    num_hidden_layers=self.num_hidden_layers, num_labels=self.num_labels)

    def __repr__(self):
        return f"TimesformerConfig({json.dumps(self.to_dict())})"


class TimesformerForVideoClassification(torch.nn.Module):
    """fp32 master parameters in HF naming (state_dict compatible with transformers'
    `TimesformerForVideoClassification`), bf16/fp32 packed device copies for the kernels."""

    def __init__(self, config: TimesformerConfig):
        super().__init__()
        self.config = config
        c = config
        if c.hidden_size // c.num_attention_heads != 64:
            raise ValueError("libvclip attention supports head_dim 64 only")
        if c.attention_type != "divided_space_time":
            raise ValueError("only attention_type='divided_space_time' (the reference's K400 checkpoint) is built")
        self.params = torch.nn.ParameterDict()
        shapes = timesformer_param_shapes(c.as_shape_cfg())
        self._names = list(shapes.keys())
        self.kernel_events = None  # list: HIP events around each spatial-attention launch (bench.py)
        self.concurrent_streams = None  # n > 1: the inference batch split over n HIP streams
        self.split_sizes = None  # clips per stream part (streams.run_split); None = as even as possible
        # tile config of the two 768 x 768 bf16-output projections per layer (temporal dense, spatial
        # output): the 128x128 kernel (cfg 5), not vc_gemm's pick (the persistent 256x256 kernel,
        # 297 tiles = 1.16 rounds of 256 CUs at B=16): 37.9 vs 46.9 us at M = 25344 and 24.7 vs 25.4
        # at the two-stream M = 12800 (tools/ab_gemm_cfg.py, round 3); None: vc_gemm's pick
        self.proj_cfg = 5
        # per-GEMM tile config overrides {"qkv_temporal" | "qkv_spatial" | "fc1" | "fc2": cfg} (A/B hook)
        self.gemm_cfg = {}
        self._streams = None
        self._split_out = {}
        # True: the inference forward is captured once per input / configuration into a hipGraph and
        # replayed (streams.GraphReplay); bit-identical logits
        self.graph_replay = False
        self._graphs = None
        for name, shape in shapes.items():
            self.params[name.replace(".", "__")] = torch.nn.Parameter(torch.zeros(shape))
        self._packed = None
        self._ws = {}
        self._ws_used = []

    def state_dict(self, *a, **k):
        return OrderedDict((n, self.params[n.replace(".", "__")].detach()) for n in self._names)

    def load_state_dict(self, sd, strict: bool = True):
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
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

    def P(self, name):
        return self.params[name.replace(".", "__")]

    def _weights_version(self):
        from . import vivit_train
        return (vivit_train.MASTER_EPOCH[0], sum(p._version for p in self.params.values()))

    def _pack(self, device):
        ver = self._weights_version()  # the fused AdamW updates in place without bumping _version
        if self._packed is not None and self._packed["device"] == device and self._packed["version"] == ver:
            return self._packed
        c = self.config
        bf, f32 = torch.bfloat16, torch.float32
        P = lambda n: self.P(n).detach().to(device=device, dtype=f32)  # noqa: E731
        D, T = c.hidden_size, c.num_frames
        e = "timesformer.embeddings."
        pk = {"device": device, "version": ver}
        pk["w_emb"] = P(e + "patch_embeddings.projection.weight").reshape(D, -1).to(bf).contiguous()
        pk["b_emb"] = P(e + "patch_embeddings.projection.bias").contiguous()
        pos = P(e + "position_embeddings").reshape(-1, D)
        tim = P(e + "time_embeddings").reshape(-1, D)
        # EMBED epilogue table: row p*T + t = pos[1 + p] + time[t] (patch-major, time-minor)
        pk["pos_time"] = (pos[1:, None, :] + tim[None, :T, :]).reshape(-1, D).contiguous()
        pk["pos"] = pos.contiguous()
        pk["cls"] = P(e + "cls_token").reshape(D).contiguous()
        qs = (D // c.num_attention_heads) ** -0.5 * ops.LOG2E  # softmax scale * log2(e) folded into q

        def qkv(prefix):
            w = P(prefix + "attention.qkv.weight").clone()
            b = P(prefix + "attention.qkv.bias").clone()
            w[:D] *= qs
            b[:D] *= qs
            return w.to(bf).contiguous(), b.contiguous()

        layers = []
        for i in range(c.num_hidden_layers):
            p = f"timesformer.encoder.layer.{i}."
            L = {}
            for ln, key in (("temporal_layernorm", "lnt"), ("layernorm_before", "ln1"), ("layernorm_after", "ln2")):
                L[key + "_g"] = P(p + ln + ".weight").contiguous()
                L[key + "_b"] = P(p + ln + ".bias").contiguous()
            L["w_qkv_t"], L["b_qkv_t"] = qkv(p + "temporal_attention.")
            wto, bto = P(p + "temporal_attention.output.dense.weight"), P(p + "temporal_attention.output.dense.bias")
            wtd, btd = P(p + "temporal_dense.weight"), P(p + "temporal_dense.bias")
            L["w_t"] = (wtd.double() @ wto.double()).to(bf).contiguous()
            L["b_t"] = (wtd.double() @ bto.double() + btd.double()).to(f32).contiguous()
            L["w_qkv_s"], L["b_qkv_s"] = qkv(p + "attention.")
            L["w_o"] = P(p + "attention.output.dense.weight").to(bf).contiguous()
            L["b_o"] = P(p + "attention.output.dense.bias").contiguous()
            L["w_1"] = P(p + "intermediate.dense.weight").to(bf).contiguous()
            L["b_1"] = P(p + "intermediate.dense.bias").contiguous()
            L["w_2"] = P(p + "output.dense.weight").to(bf).contiguous()
            L["b_2"] = P(p + "output.dense.bias").contiguous()
            layers.append(L)
        pk["layers"] = layers
        pk["lnf_g"] = P("timesformer.layernorm.weight").contiguous()
        pk["lnf_b"] = P("timesformer.layernorm.bias").contiguous()
        pk["w_cls"] = P("classifier.weight").contiguous()
        pk["b_cls"] = P("classifier.bias").contiguous()
        self._packed = pk
        return pk

    def geometry(self, B):
        c = self.config
        P = (c.image_size // c.patch_size) ** 2
        T = c.num_frames
        S = 1 + P * T
        Mpad = _round_up(max(B * S, B * T * (1 + P)) + 128, 256)
        Memb = _round_up(B * P * T, 128)
        return P, T, S, Mpad, Memb

    def _workspace(self, B, device, part: int = 0):
        key = (B, str(device), part)
        if key in self._ws:
            ws = self._ws[key]
            if not any(w is ws for w in self._ws_used):
                self._ws_used.append(ws)
            return ws
        if len(self._ws) >= 8:
            self._ws = {}
        c = self.config
        D, I = c.hidden_size, c.intermediate_size
        P, T, S, Mpad, Memb = self.geometry(B)
        bf = torch.bfloat16
        z = lambda *s, dt=bf: torch.zeros(s, dtype=dt, device=device)  # noqa: E731
        ws = dict(A_emb=z(Memb, c.num_channels * c.patch_size * c.patch_size), X=z(Mpad, D, dt=torch.float32),
                  Hc=z(Mpad, D), Hf=z(Mpad, D), QKV=z(Mpad, 3 * D), O=z(Mpad, D), Yb=z(Mpad, D), Hd=z(Mpad, I),
                  logits=z(B, c.num_labels, dt=torch.float32))
        self._ws[key] = ws
        self._ws_used.append(ws)
        return ws

    def forward(self, pixel_values: torch.Tensor = None, labels: torch.Tensor = None, **kw):
        """HF call convention.  In training mode with autograd enabled (the reference's train loop,
        timesformer/timesformer_classifier/trainers/trainer.py:165-174) the logits carry the graph of
        the HIP train step (_forward_train); otherwise the fused inference path runs."""
        if pixel_values is None:
            raise ValueError("pixel_values required")
        if pixel_values.device.type != "cuda":
            raise RuntimeError("TimesformerForVideoClassification (vclip_amd) runs on the GPU only")
        x = pixel_values.contiguous().float() if pixel_values.dtype != torch.float32 else pixel_values.contiguous()
        if self.training and torch.is_grad_enabled():
            logits = self._forward_train(x)
        else:
            with torch.no_grad():
                logits = self.forward_logits(x)
        loss = None
        if labels is not None:
            loss = torch.nn.functional.cross_entropy(logits, labels.to(logits.device))
        return ClassifierOutput(logits, loss)

    def forward_logits(self, pix: torch.Tensor) -> torch.Tensor:
        """logits f32 [B, labels] (a workspace buffer, overwritten by the next call); with
        `concurrent_streams = n > 1` the batch is split over n HIP streams (vclip_amd.streams)."""
        c = self.config
        B, T, C, H, W = pix.shape
        if T != c.num_frames or H != c.image_size or W != c.image_size or C != c.num_channels:
            raise ValueError(f"pixel_values {tuple(pix.shape)} do not match config "
                             f"(T={c.num_frames}, C={c.num_channels}, {c.image_size}^2)")
        if (self.graph_replay and self.kernel_events is None and not streams.serial()
                and not torch.cuda.is_current_stream_capturing()):
            from .streams import GraphReplay
            if self._graphs is None:
                self._graphs = GraphReplay()
            key = (pix.data_ptr(), tuple(pix.shape), tuple(pix.stride()), pix.dtype, self.concurrent_streams, None if self.split_sizes is None else tuple(self.split_sizes), self.proj_cfg,
                   tuple(sorted(self.gemm_cfg.items())),
                   str(pix.device), self._weights_version())
            return self._graphs.run(key, pix, self._forward_eager,
                                    keep=lambda: (self._packed, tuple(self._ws_used)))
        return self._forward_eager(pix)

    def _forward_eager(self, pix: torch.Tensor) -> torch.Tensor:
        self._ws_used = []  # the workspaces this forward addresses (a captured graph keeps exactly these)
        c = self.config
        B = pix.shape[0]
        ns = max(1, min(int(self.concurrent_streams or 1), B))
        if ns == 1:
            return self._forward_part(pix, 0)
        from .streams import run_split
        return run_split(self, pix, ns, self._forward_part, c.num_labels, prepare=lambda: self._pack(pix.device))

    def _forward_part(self, pix: torch.Tensor, part: int, out=None) -> torch.Tensor:
        c = self.config
        B = pix.shape[0]
        pk = self._pack(pix.device)
        ws = self._workspace(B, pix.device, part)
        P, T, S, Mpad, Memb = self.geometry(B)
        Hn = c.num_attention_heads
        eps = c.layer_norm_eps
        X, Hc, Hf, QKV, O, Yb, Hd = (ws[k] for k in ("X", "Hc", "Hf", "QKV", "O", "Yb", "Hd"))
        pc = c.patch_size
        D, I = c.hidden_size, c.intermediate_size
        Kemb = c.num_channels * pc * pc
        tm = ops.timed
        # algorithmic work per launch for an installed ops.OpRecorder: clip rows B*S (temporal
        # branch and MLP), frame rows B*T*(1+P) (spatial branch), no padding
        Mc, Mf = B * S, B * T * (1 + P)
        tm("im2col_kernel", "im2col", B * T * (c.num_channels * c.image_size ** 2 * 4 + P * Kemb * 2), "byte",
           ops.tubelet_im2col, pix, (1, pc, pc), ws["A_emb"], order="patch_major")
        ops.gemm(ws["A_emb"], pk["w_emb"], pk["b_emb"], "embed_f32", X, aux=pk["pos_time"], group=P * T,
                 group_stride=S, group_offset=1, m=Memb, flop=2.0 * B * P * T * D * Kemb, op="embed")
        ops.cls_init(pk["cls"], pk["pos"], X, B, S)
        act = "bias_gelu_erf" if c.hidden_act == "gelu" else "bias_gelu_tanh"
        scale = 1.0 / math.sqrt(c.hidden_size // Hn)
        pcfg = -1 if self.proj_cfg is None else self.proj_cfg
        gc = self.gemm_cfg
        for L in pk["layers"]:
            # temporal branch (clip layout)
            tm("layernorm_kernel", "layernorm", Mc * D * 6, "byte", ops.layernorm, X, L["lnt_g"], L["lnt_b"], eps, Hc,
               m=B * S)
            ops.gemm(Hc, L["w_qkv_t"], L["b_qkv_t"], "bias", QKV, cfg=gc.get("qkv_temporal", -1), flop=2.0 * Mc * 3 * D * D, op="qkv_temporal")
            tm("temporal_attn_lds_kernel", "temporal_attention", 4.0 * T * T * 64 * Hn * B * P, "flop",
               ops.temporal_attention, QKV, B, P, T, Hn, scale, O, q_prescaled=True)
            ops.gemm(O, L["w_t"], L["b_t"], "bias", Yb, cfg=pcfg, flop=2.0 * Mc * D * D, op="proj_temporal")
            # spatial branch (frame layout): X += temporal output, LayerNorm in the frame layout
            tm("tsf_add_ln_kernel", "add_layernorm", Mc * D * (4 + 2 + 4) + Mf * D * 2, "byte",
               ops.divided_add_layernorm, X, Yb, B, P, T, L["ln1_g"], L["ln1_b"], eps, "temporal_to_spatial", Hf)
            ops.gemm(Hf, L["w_qkv_s"], L["b_qkv_s"], "bias", QKV, cfg=gc.get("qkv_spatial", -1), flop=2.0 * Mf * 3 * D * D, op="qkv_spatial")
            ev = self.kernel_events
            if ev is not None:  # recorded on the current stream, the one the kernel runs on
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            tm("attn_short_d64_kernel", "spatial_attention", 4.0 * (1 + P) * (1 + P) * 64 * Hn * B * T, "flop",
               ops.attention, QKV, B * T, 1 + P, Hn, scale, O, q_prescaled=True)
            if ev is not None:
                e1.record()
                # flop, algorithmic bytes (q, k, v read and the output written once: 4 x 64 x 2 B
                # per token-head)
                ev.append((e0, e1, 4.0 * (1 + P) * (1 + P) * 64 * Hn * B * T, 512.0 * (1 + P) * Hn * B * T))
            ops.gemm(O, L["w_o"], L["b_o"], "bias", Yb, cfg=pcfg, flop=2.0 * Mf * D * D, op="o_proj")
            # MLP (clip layout)
            tm("tsf_add_ln_kernel", "add_layernorm", Mf * D * 2 + Mc * D * (4 + 4 + 2), "byte",
               ops.divided_add_layernorm, X, Yb, B, P, T, L["ln2_g"], L["ln2_b"], eps, "spatial_to_mlp", Hc)
            ops.gemm(Hc, L["w_1"], L["b_1"], act, Hd, cfg=gc.get("fc1", -1), flop=2.0 * Mc * I * D, op="fc1")
            ops.gemm(Hd, L["w_2"], L["b_2"], "bias_resid_f32", X, cfg=gc.get("fc2", -1), flop=2.0 * Mc * D * I, op="fc2")
        return ops.cls_head(X, B, S, pk["lnf_g"], pk["lnf_b"], eps, pk["w_cls"], pk["b_cls"],
                            out=ws["logits"] if out is None else out)


    def _forward_train(self, pix: torch.Tensor) -> torch.Tensor:
        """The TimeSformer forward (TF5/models/timesformer/modeling_timesformer.py:67-145, 332-398,
        oracle/timesformer_ref.py) as autograd ops over the HIP kernels (vclip_amd/autograd_ops.py):
        bf16 MFMA GEMMs with fp32 accumulation on the fp32 master weights, fp32 residual stream,
        exact GELU, flash spatial attention, VALU temporal attention; layout glue in torch."""
        from . import autograd_ops as A
        c = self.config
        B, T, C, H, W = pix.shape
        if T != c.num_frames or H != c.image_size or W != c.image_size or C != c.num_channels:
            raise ValueError(f"pixel_values {tuple(pix.shape)} do not match config")
        if c.hidden_act != "gelu":
            raise NotImplementedError("train step: hidden_act 'gelu' (TimeSformer's) only")
        D, Hn, eps, pc = c.hidden_size, c.num_attention_heads, c.layer_norm_eps, c.patch_size
        P = (c.image_size // pc) ** 2
        S = 1 + P * T
        e = "timesformer.embeddings."
        M = B * P * T
        a_emb = torch.zeros(_round_up(M, 128), C * pc * pc, dtype=torch.bfloat16, device=pix.device)
        ops.tubelet_im2col(pix, (1, pc, pc), a_emb, order="patch_major")  # rows (b, p, t)
        emb = A.linear(a_emb[:M], self.P(e + "patch_embeddings.projection.weight").reshape(D, -1),
                       self.P(e + "patch_embeddings.projection.bias"), out_f32=True)
        pos = self.P(e + "position_embeddings").reshape(-1, D)
        tim = self.P(e + "time_embeddings").reshape(-1, D)[:T]
        emb = emb.reshape(B, P, T, D) + pos[1:].reshape(1, P, 1, D) + tim.reshape(1, 1, T, D)
        cls = (self.P(e + "cls_token").reshape(1, 1, D) + pos[0].reshape(1, 1, D)).expand(B, 1, D)
        x = torch.cat([cls, emb.reshape(B, P * T, D)], 1)  # [B, S, D] patch-major, time-minor
        qs = (D // Hn) ** -0.5 * ops.LOG2E
        for i in range(c.num_hidden_layers):
            p = f"timesformer.encoder.layer.{i}."
            W_ = lambda n: self.P(p + n)  # noqa: E731
            # temporal branch on the clip layout (CLS rows computed and discarded, as inference)
            h = A.layer_norm(x.reshape(B * S, D), W_("temporal_layernorm.weight"), W_("temporal_layernorm.bias"), eps)
            qkv = A.linear(h, W_("temporal_attention.attention.qkv.weight"), W_("temporal_attention.attention.qkv.bias"),
                           qrows=D, qscale=qs)
            o = A.temporal_attention(qkv, B, P, T, Hn)
            a = A.linear(o, W_("temporal_attention.output.dense.weight"), W_("temporal_attention.output.dense.bias"))
            rt = A.linear(a, W_("temporal_dense.weight"), W_("temporal_dense.bias"), out_f32=True).reshape(B, S, D)
            te = x[:, 1:] + rt[:, 1:]
            # spatial branch: B*T sequences of CLS + P patches
            init_cls = x[:, :1]
            sp = te.reshape(B, P, T, D).permute(0, 2, 1, 3).reshape(B * T, P, D)
            sp = torch.cat([init_cls.expand(B, T, D).reshape(B * T, 1, D), sp], 1)
            h = A.layer_norm(sp.reshape(B * T * (1 + P), D), W_("layernorm_before.weight"), W_("layernorm_before.bias"),
                             eps)
            qkv = A.linear(h, W_("attention.attention.qkv.weight"), W_("attention.attention.qkv.bias"), qrows=D,
                           qscale=qs)
            o = A.attention(qkv, B * T, 1 + P, Hn)
            y = A.linear(o, W_("attention.output.dense.weight"), W_("attention.output.dense.bias"),
                         out_f32=True).reshape(B * T, 1 + P, D)
            cls_res = y[:, 0].reshape(B, T, D).mean(1, keepdim=True)
            res = y[:, 1:].reshape(B, T, P, D).permute(0, 2, 1, 3).reshape(B, P * T, D)
            x = torch.cat([init_cls + cls_res, te + res], 1)
            # MLP
            h = A.layer_norm(x.reshape(B * S, D), W_("layernorm_after.weight"), W_("layernorm_after.bias"), eps)
            g = A.gelu_erf(A.linear(h, W_("intermediate.dense.weight"), W_("intermediate.dense.bias")))
            x = x + A.linear(g, W_("output.dense.weight"), W_("output.dense.bias"), out_f32=True).reshape(B, S, D)
        return A.cls_head(x.reshape(B * S, D), self.P("timesformer.layernorm.weight"),
                          self.P("timesformer.layernorm.bias"), self.P("classifier.weight"), self.P("classifier.bias"),
                          B, S, eps)


def create_model(model_name="facebook/timesformer-base-finetuned-k400", num_classes=2, class_labels=None,
                 num_frames=8, device="cuda", logger=None, weights_seed: int = 0):
    """Drop-in for timesformer/timesformer_classifier/models/timesformer_model.py:4-53.

    The reference loads `TimesformerConfig.from_pretrained(model_name)` + K400 weights
    (`ignore_mismatched_sizes=True` re-initialises the head, and the time embeddings when
    num_frames != 8).  No network here: the TimeSformer-B architecture is built with seeded
    synthetic weights (vclip_amd.weights) unless a checkpoint is loaded afterwards.
    """
    class_labels = class_labels or ["non-referral", "referral"]
    id2label = {i: l for i, l in enumerate(class_labels)}
    cfg = TimesformerConfig(num_frames=num_frames, id2label=id2label, label2id={l: i for i, l in id2label.items()},
                            num_classes=num_classes, video_size=[num_frames, 224, 224])
    if logger:
        logger.info(f"Creating TimeSformer model based on {model_name} (num_frames={num_frames}) on {device}")
    model = TimesformerForVideoClassification(cfg)
    from .weights import make_timesformer_weights
    model.load_state_dict(make_timesformer_weights(cfg.as_shape_cfg(), seed=weights_seed))
    return model.to(device) if device else model
