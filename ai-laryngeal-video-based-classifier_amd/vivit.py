"""ViViT-B/16x2 video classifier on the libvclip.so kernels — drop-in for the reference's
`create_model` (vivit_transformer/vivit_classifier/models/vivit_model.py:4-52), which
returns an HF `VivitForVideoClassification` called as `model(pixel_values=...)` and
read through `.logits` (vivit_transformer/vivit_classifier/trainers/trainer.py:141-142,
vivit_transformer/inference.py:192-193).

Device data layout (one forward of B clips, S = 1 + (T/2)(H/16)(W/16) tokens):
  rows r = b*S + s, padded to Mpad = roundup(B*S + 128, 256) so every GEMM runs on
  whole 128-row tiles and attention can read a full 64-key tile past each clip's end;
  residual stream X   f32  [Mpad, D]          (fp32 residual adds, as the fp32 reference)
  LN output Y         bf16 [Mpad, D]
  fused q|k|v         bf16 [Mpad, 3D]
  attention out O     bf16 [Mpad, D]
  MLP hidden          bf16 [Mpad, 4D]
Weights are packed once per device: bf16 [N, K] (nn.Linear layout), q|k|v concatenated,
fp32 biases / LayerNorm / position table / classifier.
"""
from __future__ import annotations

import functools
import json
import math
from collections import OrderedDict

import numpy as np
import torch

from . import ops, streams
from .streams import GraphReplay
from .vivit_train import FlatLayout, TrainEngine, VivitTrainFn
from .weights import vivit_param_shapes


class VivitConfig:
    """Minimal stand-in for transformers.VivitConfig (fields the path and the reference's
    checkpoint dict use: trainer.py:281-299 saves config.to_dict(), id2label, label2id)."""

    defaults = dict(image_size=224, num_frames=32, tubelet_size=[2, 16, 16], num_channels=3, hidden_size=768,
                    num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072, hidden_act="gelu_fast",
                    hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, initializer_range=0.02,
                    layer_norm_eps=1e-6, qkv_bias=True, model_type="vivit")

    def __init__(self, **kw):
        d = dict(self.defaults)
        d.update(kw)
        id2label = d.pop("id2label", None) or {0: "LABEL_0", 1: "LABEL_1"}
        self.id2label = {int(k): v for k, v in id2label.items()}
        self.label2id = d.pop("label2id", None) or {v: k for k, v in self.id2label.items()}
        d.pop("num_labels", None)
        for k, v in d.items():
            setattr(self, k, v)
        self.tubelet_size = list(self.tubelet_size)

    @property
    def num_labels(self):
        return len(self.id2label)

    def to_dict(self):
        d = {k: getattr(self, k) for k in self.defaults}
        d["id2label"] = {str(k): v for k, v in self.id2label.items()}
        d["label2id"] = dict(self.label2id)
        return d

    @classmethod
    def from_dict(cls, d):
        return cls(**d)

    def as_shape_cfg(self):
        return dict(hidden_size=self.hidden_size, intermediate_size=self.intermediate_size,
                    tubelet_size=self.tubelet_size, num_channels=self.num_channels, num_frames=self.num_frames,
                    image_size=self.image_size, num_hidden_layers=self.num_hidden_layers,
                    num_labels=self.num_labels)

    def __repr__(self):
        return f"VivitConfig({json.dumps(self.to_dict())})"


class ClassifierOutput:
    """Mimics the `.logits` / `.loss` access of transformers' ImageClassifierOutput."""

    def __init__(self, logits, loss=None):
        self.logits = logits
        self.loss = loss

    def __getitem__(self, i):
        return (self.loss, self.logits)[i] if self.loss is not None else (self.logits,)[i]


# Clips per stream part where an uneven split measured faster than the even one (model.split_sizes
# overrides).  ViViT-B B = 8 on two streams: 5 + 3 vs 4 + 4, +2.2 / +1.8 % in two interleaved
# A/Bs on different boxes (tools/ab_split_sizes.py, profiles/r05_split_sizes.txt; 3 + 5 -0.8 %,
# 6 + 2 -0.9 %): the 5-clip part's 1500 attention workgroups fill 2.93 rounds of the 512
# two-per-CU slots where 4 clips' 1200 fill 2.34, and the parts pad 25344 token rows to the
# 256-row GEMM tiles instead of 25600.  The larger part goes first (its stream starts first).
# TimeSformer-B (10 + 6, 9 + 7) and ResNet3D (3 + 1) measured slower than even.
SPLIT_DEFAULT = {(8, 2): (5, 3)}


def _round_up(x, m):
    return (x + m - 1) // m * m


class VivitForVideoClassification(torch.nn.Module):
    """fp32 master parameters in HF naming (state_dict compatible with transformers-5
    `VivitForVideoClassification`), bf16/fp32 packed device copies for the kernels."""

    def __init__(self, config: VivitConfig):
        super().__init__()
        self.config = config
        c = config
        if c.hidden_size // c.num_attention_heads != 64:
            raise ValueError("libvclip attention supports head_dim 64 only")
        self.params = torch.nn.ParameterDict()
        shapes = vivit_param_shapes(c.as_shape_cfg())
        self._names = list(shapes.keys())
        for name, shape in shapes.items():
            self.params[name.replace(".", "__")] = torch.nn.Parameter(torch.zeros(shape))
        self._layout = FlatLayout(c, shapes)
        self._flat = None      # fp32 masters, one device buffer (params are views), built for training
        self._gflat = None     # gradients, same layout (p.grad are views)
        self._gscratch = None  # backward target when gradients accumulate across calls
        self._engine = None
        self.grad_ready_hooks = []  # fn(stage, start, end, gflat): a slice of gflat is final (enqueued)
        self._packed = None
        self._ws = {}
        self._ws_used = []
        self._streams = None
        self.concurrent_streams = None  # None / 1: one stream; n > 1: batch split over n HIP streams
        # HIP stream priority per part (lower is higher) of the eager forward's part streams, an A/B hook;
        # None: the stream set streams.part_streams timed fastest on the first call.  Under graph replay
        # the part graphs run on the set streams.GraphReplay._tune timed fastest; profiles/r06_hwq.txt
        self.stream_priorities = None
        # clips per stream part (A/B hook; must sum to the batch): None = as even as possible
        self.split_sizes = None
        self.last_streams = 1
        self.kernel_events = None
        # True: the inference forward is captured once per input / configuration into a hipGraph
        # and replayed (streams.GraphReplay); bit-identical logits
        self.graph_replay = False
        self._graphs = GraphReplay()
        # per-GEMM tile config override {"qkv" | "o_proj" | "fc1" | "fc2": vc_gemm cfg} (None / absent:
        # vc_gemm's own pick) and the GEMM / LayerNorm row count: "pad" = every padded row (Mpad),
        # "tight" = B*S rounded up to the tile height (the padding rows keep their initial zeros)
        self.gemm_cfg = {}
        self.rows = "pad"
        # 16-bit operand type of the inference forward: bf16 (the benchmarked configuration) or
        # torch.float16 (same kernels and MFMA rate, logits ~6x closer to the fp32 reference;
        # DESIGN.md §5.5).  The train step (vivit_train.py) is bf16 either way.
        self.compute_dtype = torch.bfloat16
        # fp16 build only: the patch embedding and the first `precise_layers` layers' GEMMs take split
        # operands -- weights as fp16 high + low parts (and the pixels too in the embedding) through
        # vc_gemm_h16_wrap, A.W_hi + A.W_lo in one fp32 chain.  The fp16 build's logit error is set by
        # the weight rounding of the first layers (tests/analysis/w_probe.py: all weights fp32 3.8e-4, the
        # embedding + layer 0 4.3e-4, vs 1.25e-3 all fp16 on the bench's 8 clips).
        self.precise_layers = 0
        # ... and which GEMMs: "embed" (pixels and weights split: three products) or "embed_w" (weights
        # only: A.W_hi + A.W_lo), and layer 0's "qkv" / "o_proj" / "fc1" / "fc2".  Default: the
        # embedding's weights and layer 0's q|k|v -- logit error 6.3e-4 on 4 of the bench's clips vs 6.7e-4
        # with the pixels and all of layer 0 split too, at less than half the extra MFMA work (957 vs 926
        # clips/s, bf16 982: tests/test_fp16_gpu.py, profiles/r05_fp16_clock.json)
        self.precise_ops = ("embed_w", "qkv")

    # ---- state dict in HF naming ---------------------------------------------------
    def hf_state_dict(self):
        return OrderedDict((n, self.params[n.replace(".", "__")]) for n in self._names)

    def state_dict(self, *a, **k):  # noqa: D401 - HF key names, like the reference's model
        return OrderedDict((n, p.detach()) for n, p in self.hf_state_dict().items())

    def load_state_dict(self, sd, strict: bool = True):
        from .checkpoint import convert_state_dict
        sd = convert_state_dict(sd)
        missing = [n for n in self._names if n not in sd]
        unexpected = [k for k in sd if k not in self._names]
        if strict and (missing or unexpected):
            raise KeyError(f"load_state_dict: missing={missing[:5]} unexpected={unexpected[:5]}")
        with torch.no_grad():
            for n in self._names:
                if n in sd:
                    v = sd[n]
                    v = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
                    self.params[n.replace(".", "__")].copy_(v.reshape(self.params[n.replace(".", "__")].shape))
        self._packed = None
        return missing, unexpected

    def P(self, name):
        return self.params[name.replace(".", "__")]

    def _param_list(self):
        return [self.P(n) for n in self._names]

    def _apply(self, fn, *args, **kwargs):  # .to() / .cuda(): parameters move one by one
        out = super()._apply(fn, *args, **kwargs)
        self._flat = self._gflat = self._gscratch = self._engine = None
        self._packed = None
        self._ws = {}
        self._streams = None
        self._graphs.clear()
        return out

    # ---- training (vclip_amd/vivit_train.py) --------------------------
    def _ensure_flat(self, device):
        """Move the fp32 masters into one flat device buffer, parameters becoming views of it
        (the same Parameter objects, so an optimizer built earlier keeps working)."""
        if self._flat is not None and self._flat.device == device:
            return
        flat = torch.zeros(self._layout.total, dtype=torch.float32, device=device)
        with torch.no_grad():
            for n in self._names:
                v = self._layout.view(flat, n)
                v.copy_(self.P(n).detach().reshape(v.shape))
                self.P(n).data = v
                # the optimizer's one-launch path needs to know that a parameter list covers the
                # whole layout (its alignment gaps stay zero in both buffers: AdamW keeps them 0)
                self.P(n)._vc_flat_layout = (self._layout.total, len(self._names))
        self._flat = flat
        self._gflat = torch.zeros_like(flat)
        self._gscratch = None
        self._engine = None

    def _train_engine(self, B, device):
        self._ensure_flat(device)
        if self._engine is None or self._engine.B != B or self._engine.device != device:
            self._engine = None
            self._engine = TrainEngine(self, B, device)
        return self._engine

    def _run_backward(self, eng, dlogits):
        params = self._param_list()
        accumulate = any(p.grad is not None for p in params)
        if not accumulate:
            target = self._gflat
        else:
            if self._gscratch is None:
                self._gscratch = torch.zeros_like(self._gflat)
            target = self._gscratch

        stages = []

        def ready(stage, start, end):
            if not accumulate:
                for h in self.grad_ready_hooks:
                    h(stage, start, end, target)
            else:
                stages.append((stage, start, end))

        if accumulate and self.grad_ready_hooks:
            g0 = self._gflat.untyped_storage().data_ptr()
            if any(p.grad is not None and p.grad.untyped_storage().data_ptr() != g0 for p in params):
                raise RuntimeError("gradient accumulation with grad_ready_hooks (data-parallel all-reduce) needs "
                                   "every .grad to be the model's own flat-buffer view; zero_grad(set_to_none=True) "
                                   "or leave .grad as the backward set it")
        eng.backward(dlogits, target, ready)
        lay = self._layout
        if not accumulate:
            for n, p in zip(self._names, params):
                p.grad = lay.view(self._gflat, n)
            return
        for n, p in zip(self._names, params):
            g = lay.view(target, n)
            if p.grad is None:
                p.grad = lay.view(self._gflat, n).copy_(g)
            else:
                p.grad.add_(g)
        # accumulated gradients: the hooks (e.g. GradAllReduce) see the summed flat buffer, stage
        # by stage in backward order once the sum is complete -- as DDP reduces the accumulated
        # .grad on every backward (the average of (mean + local) is mean + mean)
        for stage, start, end in stages:
            for h in self.grad_ready_hooks:
                h(stage, start, end, self._gflat)

    def _weights_version(self):
        from . import vivit_train
        return (vivit_train.MASTER_EPOCH[0], sum(p._version for p in self._param_list()))

    # ---- device packing ----------------------------------------------------------
    def _pack(self, device):
        ver = self._weights_version()
        bf = self.compute_dtype
        if bf not in (torch.bfloat16, torch.float16):
            raise ValueError(f"compute_dtype must be torch.bfloat16 or torch.float16, not {bf}")
        npre = self.precise_layers if bf == torch.float16 else 0
        pops = tuple(sorted(self.precise_ops)) if npre > 0 else ()
        if not set(pops) <= {"embed", "embed_w", "qkv", "o_proj", "fc1", "fc2"} or {"embed", "embed_w"} <= set(pops):
            raise ValueError(f"precise_ops must name embed | embed_w and q|k|v / o_proj / fc1 / fc2, not {self.precise_ops}")
        if (self._packed is not None and self._packed["device"] == device and self._packed["version"] == ver
                and self._packed["dtype"] == bf and self._packed["precise"] == npre and self._packed["pops"] == pops):
            return self._packed
        c = self.config
        f32 = torch.float32
        P = lambda n: self.P(n).detach().to(device)  # noqa: E731
        D = c.hidden_size
        kt, kh, kw = c.tubelet_size
        pk = {"device": device, "version": ver, "dtype": bf, "precise": npre, "pops": pops}

        def split(w, emb=False):
            # [W_hi | W_lo] (embedding: [W_hi | W_hi | W_lo] against [A_hi | A_lo] with A wrapping)
            w = w.float()
            hi = w.to(torch.float16)
            lo = (w - hi.float()).to(torch.float16)
            return torch.cat([hi, hi, lo] if emb else [hi, lo], dim=1).contiguous()

        pk["w_emb"] = P("vivit.embeddings.patch_embeddings.projection.weight").reshape(D, -1).to(bf).contiguous()
        if "embed" in pops or "embed_w" in pops:
            pk["w_emb_split"] = split(P("vivit.embeddings.patch_embeddings.projection.weight").reshape(D, -1),
                                      emb="embed" in pops)
        pk["b_emb"] = P("vivit.embeddings.patch_embeddings.projection.bias").to(f32).contiguous()
        pk["pos"] = P("vivit.embeddings.position_embeddings").reshape(-1, D).to(f32).contiguous()
        pk["cls"] = P("vivit.embeddings.cls_token").reshape(D).to(f32).contiguous()
        layers = []
        for i in range(c.num_hidden_layers):
            p = f"vivit.layers.{i}."
            L = {}
            L["ln1_g"] = P(p + "layernorm_before.weight").contiguous()
            L["ln1_b"] = P(p + "layernorm_before.bias").contiguous()
            L["ln2_g"] = P(p + "layernorm_after.weight").contiguous()
            L["ln2_b"] = P(p + "layernorm_after.bias").contiguous()
            # softmax scale * log2(e) folded into the q projection (fp32 master -> one bf16 rounding),
            # so the attention kernel's exp2 argument comes straight out of the QK^T MFMA
            qs = (D // c.num_attention_heads) ** -0.5 * ops.LOG2E
            L["w_qkv"] = torch.cat([P(p + "attention.q_proj.weight") * qs, P(p + "attention.k_proj.weight"),
                                    P(p + "attention.v_proj.weight")]).to(bf).contiguous()
            L["b_qkv"] = torch.cat([P(p + "attention.q_proj.bias") * qs, P(p + "attention.k_proj.bias"),
                                    P(p + "attention.v_proj.bias")]).contiguous()
            L["w_o"] = P(p + "attention.o_proj.weight").to(bf).contiguous()
            L["b_o"] = P(p + "attention.o_proj.bias").contiguous()
            L["w_1"] = P(p + "mlp.fc1.weight").to(bf).contiguous()
            L["b_1"] = P(p + "mlp.fc1.bias").contiguous()
            L["w_2"] = P(p + "mlp.fc2.weight").to(bf).contiguous()
            L["b_2"] = P(p + "mlp.fc2.bias").contiguous()
            if i < npre:
                sp = {}
                if "qkv" in pops:
                    sp["w_qkv"] = split(torch.cat([P(p + "attention.q_proj.weight") * qs,
                                                   P(p + "attention.k_proj.weight"), P(p + "attention.v_proj.weight")]))
                if "o_proj" in pops:
                    sp["w_o"] = split(P(p + "attention.o_proj.weight"))
                if "fc1" in pops:
                    sp["w_1"] = split(P(p + "mlp.fc1.weight"))
                if "fc2" in pops:
                    sp["w_2"] = split(P(p + "mlp.fc2.weight"))
                L["split"] = sp
            layers.append(L)
        pk["layers"] = layers
        pk["lnf_g"] = P("vivit.layernorm.weight").contiguous()
        pk["lnf_b"] = P("vivit.layernorm.bias").contiguous()
        pk["w_cls"] = P("classifier.weight").to(f32).contiguous()
        pk["b_cls"] = P("classifier.bias").to(f32).contiguous()
        self._packed = pk
        return pk

    def geometry(self, B):
        c = self.config
        kt, kh, kw = c.tubelet_size
        npatch = (c.num_frames // kt) * (c.image_size // kh) * (c.image_size // kw)
        S = npatch + 1
        Mpad = _round_up(B * S + 128, 256)
        Memb = _round_up(B * npatch, 128)
        return npatch, S, Mpad, Memb

    def _workspace(self, B, device, part: int = 0):
        key = (B, str(device), part, self.compute_dtype, self.precise_layers > 0)
        if key in self._ws:
            ws = self._ws[key]
            if not any(w is ws for w in self._ws_used):
                self._ws_used.append(ws)
            return ws
        if len(self._ws) >= 8:  # (1 + 2 stream parts) x {bf16, fp16} + the split logits fit
            self._ws = {}
        c = self.config
        D, I = c.hidden_size, c.intermediate_size
        kt, kh, kw = c.tubelet_size
        npatch, S, Mpad, Memb = self.geometry(B)
        bf = self.compute_dtype
        z = lambda *s, dt=bf: torch.zeros(s, dtype=dt, device=device)  # noqa: E731
        Kemb = c.num_channels * kt * kh * kw
        precise = self.precise_layers > 0 and bf == torch.float16
        if precise:
            # the split-operand embedding runs on the 256-row ping-pong kernel (vc_gemm_h16_wrap): its A rows
            # rounded up to 256 (zero rows past B*npatch), and X 256 rows deeper so the remapped rows of that
            # padding (tokens B*S+1 .. B*S+256, values bias + pos: finite) stay inside the buffer; the layers
            # address X[:Mpad] as always
            Memb = _round_up(B * npatch, 256)
            Xe = z(Mpad + 256, D, dt=torch.float32)
        else:
            Xe = z(Mpad, D, dt=torch.float32)
        ws = dict(A_emb=z(Memb, Kemb), X=Xe[:Mpad], X_emb=Xe, Y=z(Mpad, D),
                  QKV=z(Mpad, 3 * D), O=z(Mpad, D), Hd=z(Mpad, I), logits=z(B, c.num_labels, dt=torch.float32))
        if precise:
            ws["A_emb_split"] = z(Memb, 2 * Kemb)
        self._ws[key] = ws
        self._ws_used.append(ws)
        return ws

    # ---- forward -----------------------------------------------------------------
    def forward(self, pixel_values: torch.Tensor = None, labels: torch.Tensor = None, **kw):
        if pixel_values is None:
            raise ValueError("pixel_values required")
        if pixel_values.device.type != "cuda":
            raise RuntimeError("VivitForVideoClassification (vclip_amd) runs on the GPU only: move pixel_values "
                               "to cuda (the reference's `.to(device)`, trainer.py:92)")
        x = pixel_values.contiguous().float() if pixel_values.dtype != torch.float32 else pixel_values.contiguous()
        params = self._param_list()
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in params):
            logits = VivitTrainFn.apply(self, x, *params)  # forward saving activations; HIP backward
        else:
            with torch.no_grad():
                logits = self.forward_logits(x).clone()  # the workspace buffer is reused by the next call
        loss = None
        if labels is not None:
            loss = torch.nn.functional.cross_entropy(logits, labels.to(logits.device))
        return ClassifierOutput(logits, loss)

    @torch.no_grad()
    def forward_logits(self, pix: torch.Tensor) -> torch.Tensor:
        """logits f32 [B, labels] (a workspace buffer, overwritten by the next call).

        `concurrent_streams = n > 1` splits the batch over n HIP streams, each part with its own
        workspace, so one part's kernels fill the CUs another part's tail rounds and short launches
        leave idle: ViViT-B B = 8 840 -> 916 and 857 -> 911 clips/s with 2 streams on two boxes
        (tools/exp_streams.py; 3 streams 813-855).  bench.py's headline runs 2 streams; its kernel
        roofline is timed in a separate one-stream pass (under overlap a launch's event time
        includes time shared with the other stream's kernels).  Logits are bit-identical either
        way (every kernel is batch-invariant)."""
        c = self.config
        B, T, C, H, W = pix.shape
        if T != c.num_frames or H != c.image_size or W != c.image_size or C != c.num_channels:
            raise ValueError(f"pixel_values {tuple(pix.shape)} do not match config "
                             f"(T={c.num_frames}, C={c.num_channels}, {c.image_size}^2)")
        if (self.graph_replay and self.kernel_events is None and not streams.serial()
                and not torch.cuda.is_current_stream_capturing()):
            key = (pix.data_ptr(), tuple(pix.shape), tuple(pix.stride()), pix.dtype, self.concurrent_streams,
                   self.compute_dtype, self._weights_version(),
                   tuple(sorted((k, tuple(v) if isinstance(v, list) else v) for k, v in self.gemm_cfg.items())), self.rows,
                   self.precise_layers, tuple(sorted(self.precise_ops)),
                   None if self.split_sizes is None else tuple(self.split_sizes),
                   None if self.stream_priorities is None else tuple(self.stream_priorities))
            return self._graphs.run(key, pix, self._forward_eager, keep=lambda: (self._packed, tuple(self._ws_used)))
        return self._forward_eager(pix)

    def _forward_eager(self, pix: torch.Tensor) -> torch.Tensor:
        self._ws_used = []  # the workspaces this forward addresses (a captured graph keeps exactly these)
        c = self.config
        B = pix.shape[0]
        ns = self.concurrent_streams or 1
        ns = max(1, min(int(ns), B))
        self.last_streams = ns
        if ns == 1:
            self.last_split = [B]
            return self._forward_part(pix, 0)
        dev = pix.device
        key = (B, str(dev), "logits")
        if key not in self._ws:
            self._ws[key] = torch.zeros(B, c.num_labels, dtype=torch.float32, device=dev)
        logits = self._ws[key]
        cur = torch.cuda.current_stream(dev)
        # the packed weights every part reads are built on the caller's stream before the fork
        # (streams.run_split's rule): packed inside part 0 they would race parts 1..n-1
        self._pack(dev)
        bounds = streams.split_bounds(B, ns, self.split_sizes if self.split_sizes is not None
                                      else SPLIT_DEFAULT.get((B, ns)))
        self.last_split = [bounds[i + 1] - bounds[i] for i in range(ns)]
        if streams.serial():  # instrumentation: the parts one after the other on the caller's stream
            for i in range(ns):
                self._forward_part(pix[bounds[i]:bounds[i + 1]], i, out=logits[bounds[i]:bounds[i + 1]])
            return logits
        # whole parts enqueued one after the other (measured, tools/exp_streams.py: enqueueing the
        # parts layer by layer round robin ran 725 vs 911 clips/s, chaining their attention launches
        # across the streams 721, and starting part i+1 at a fixed op of part i's first layer 887-906)
        def go(sts):
            for st in sts:
                pix.record_stream(st)
            streams.fork_parts(sts, cur, [lambda i=i: self._forward_part(pix[bounds[i]:bounds[i + 1]], i,
                                                                          out=logits[bounds[i]:bounds[i + 1]])
                                          for i in range(ns)])

        # the parts' streams: on different hardware queues, the fastest of several sets timed on the first
        # call per configuration (streams.part_streams)
        self._streams = streams.part_streams(self, (B, ns, str(dev), tuple(bounds), self.compute_dtype), ns, go,
                                             dev, self.stream_priorities)
        go(self._streams)
        return logits

    def _forward_part(self, pix: torch.Tensor, part: int, out=None) -> torch.Tensor:
        c = self.config
        B = pix.shape[0]
        pk = self._pack(pix.device)
        ws = self._workspace(B, pix.device, part)
        D = c.hidden_size
        npatch, S, Mpad, Memb = self.geometry(B)
        kt_, kh_, kw_ = c.tubelet_size
        eps = c.layer_norm_eps
        X, Y, QKV, O, Hd = ws["X"], ws["Y"], ws["QKV"], ws["O"], ws["Hd"]
        # optional per-launch HIP-event timing (bench.py), recorded on this part's stream, the
        # one each kernel runs on: a list collects the attention launches only, a dict every op
        ev = self.kernel_events

        def run(name, fn, *args, **kw):
            if ev is None or (not isinstance(ev, dict) and name != "attention"):
                return fn(*args, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*args, **kw)
            e1.record()
            (ev.setdefault(name, []) if isinstance(ev, dict) else ev).append((e0, e1))
            return r

        # algorithmic work per launch for an installed ops.OpRecorder (B*S token rows, no padding)
        M = B * S
        I = c.intermediate_size
        Kemb = c.num_channels * kt_ * kh_ * kw_
        T_, H_ = c.num_frames, c.image_size
        ln_bytes = M * D * (4 + 2)
        tm = ops.timed
        if "A_emb_split" in ws and "w_emb_split" in pk and "embed_w" in pk["pops"]:
            # split weights only: A (plain fp16 im2col) wrapping against [W_hi | W_lo]
            run("im2col", tm, "im2col_kernel", "im2col", B * (T_ * c.num_channels * H_ * H_ * 4 + npatch * Kemb * 2),
                "byte", ops.tubelet_im2col, pix, c.tubelet_size, ws["A_emb"])
            run("embed", ops.gemm_wrap, ws["A_emb"], Kemb, pk["w_emb_split"], pk["b_emb"], "embed_f32", ws["X_emb"],
                aux=pk["pos"][1:], group=npatch, group_stride=S, group_offset=1, m=ws["A_emb"].shape[0],
                flop=2.0 * B * npatch * D * Kemb, op="embed")
        elif "A_emb_split" in ws and "w_emb_split" in pk:
            # split operands: [A_hi | A_lo] against [W_hi | W_hi | W_lo] (A_hi W_hi + A_lo W_hi + A_hi W_lo)
            run("im2col", tm, "im2col_kernel", "im2col", B * (T_ * c.num_channels * H_ * H_ * 4 + npatch * Kemb * 4),
                "byte", ops.patch_im2col_split, pix, c.tubelet_size, ws["A_emb_split"])
            run("embed", ops.gemm_wrap, ws["A_emb_split"], 2 * Kemb, pk["w_emb_split"], pk["b_emb"], "embed_f32",
                ws["X_emb"], aux=pk["pos"][1:], group=npatch, group_stride=S, group_offset=1,
                m=ws["A_emb_split"].shape[0],
                flop=2.0 * B * npatch * D * Kemb, op="embed")
        else:
            run("im2col", tm, "im2col_kernel", "im2col", B * (T_ * c.num_channels * H_ * H_ * 4 + npatch * Kemb * 2),
                "byte", ops.tubelet_im2col, pix, c.tubelet_size, ws["A_emb"])
            run("embed", ops.gemm, ws["A_emb"], pk["w_emb"], pk["b_emb"], "embed_f32", X, aux=pk["pos"][1:],
                group=npatch, group_stride=S, group_offset=1, m=Memb, flop=2.0 * B * npatch * D * Kemb, op="embed")
        ops.cls_init(pk["cls"], pk["pos"], X, B, S)
        act = "bias_gelu_tanh" if c.hidden_act in ("gelu_fast", "gelu_pytorch_tanh", "gelu_new") else "bias_gelu_erf"
        scale = 1.0 / math.sqrt(D // c.num_attention_heads)
        qkv_gemm = fc2_gemm = ops.gemm
        gc = self.gemm_cfg
        tight = self.rows == "tight"

        def rows(name):
            """(m, cfg) of one GEMM: every padded row, or B*S up to its tile height (256 rows for the
            256-row configs 0/3/4 and for vc_gemm's own pick, which prefers them, else 128)"""
            cfg = gc.get(name)
            if isinstance(cfg, (list, tuple)):  # one config per stream part
                cfg = cfg[part]
            if not tight:
                return None, -1 if cfg is None else cfg
            h = 128 if cfg in (5, 7, 21) else 256
            return _round_up(B * S, h), -1 if cfg is None else cfg

        m_ln = B * S if tight else None
        (m_qkv, c_qkv), (m_o, c_o), (m_1, c_1), (m_2, c_2) = rows("qkv"), rows("o_proj"), rows("fc1"), rows("fc2")
        Hn = c.num_attention_heads
        attn_flop = 4.0 * S * S * (D // Hn) * Hn * B
        for L in pk["layers"]:
            sp = L.get("split", {})  # the split-operand fp16 GEMMs (precise_layers / precise_ops): A wraps against [W_hi | W_lo]
            run("layernorm", tm, "layernorm_kernel", "layernorm", ln_bytes, "byte", ops.layernorm, X, L["ln1_g"],
                L["ln1_b"], eps, Y, m=m_ln)
            if "w_qkv" in sp:
                run("qkv", ops.gemm_wrap, Y, D, sp["w_qkv"], L["b_qkv"], "bias", QKV, flop=2.0 * M * 3 * D * D, op="qkv")
            else:
                run("qkv", qkv_gemm, Y, L["w_qkv"], L["b_qkv"], "bias", QKV, m=m_qkv, cfg=c_qkv,
                    flop=2.0 * M * 3 * D * D, op="qkv")
            run("attention", tm, "attn_fwd_d64_kernel", "attention", attn_flop, "flop", ops.attention, QKV, B, S, Hn,
                scale, O, q_prescaled=True)
            if "w_o" in sp:
                run("o_proj", ops.gemm_wrap, O, D, sp["w_o"], L["b_o"], "bias_resid_f32", X, flop=2.0 * M * D * D,
                    op="o_proj")
            else:
                run("o_proj", ops.gemm, O, L["w_o"], L["b_o"], "bias_resid_f32", X, m=m_o, cfg=c_o,
                    flop=2.0 * M * D * D, op="o_proj")
            run("layernorm", tm, "layernorm_kernel", "layernorm", ln_bytes, "byte", ops.layernorm, X, L["ln2_g"],
                L["ln2_b"], eps, Y, m=m_ln)
            if "w_1" in sp:
                run("fc1", ops.gemm_wrap, Y, D, sp["w_1"], L["b_1"], act, Hd, flop=2.0 * M * I * D, op="fc1")
            else:
                run("fc1", ops.gemm, Y, L["w_1"], L["b_1"], act, Hd, m=m_1, cfg=c_1, flop=2.0 * M * I * D, op="fc1")
            if "w_2" in sp:
                run("fc2", ops.gemm_wrap, Hd, I, sp["w_2"], L["b_2"], "bias_resid_f32", X, flop=2.0 * M * D * I,
                    op="fc2")
            else:
                run("fc2", fc2_gemm, Hd, L["w_2"], L["b_2"], "bias_resid_f32", X, m=m_2, cfg=c_2,
                    flop=2.0 * M * D * I, op="fc2")
        return ops.cls_head(X, B, S, pk["lnf_g"], pk["lnf_b"], eps, pk["w_cls"], pk["b_cls"],
                            out=ws["logits"] if out is None else out)


def create_model(model_name="google/vivit-b-16x2-kinetics400", num_classes=2, class_labels=None, num_frames=32,
                 device="cuda", logger=None, weights_seed: int = 0):
    """Drop-in for vivit_transformer/vivit_classifier/models/vivit_model.py:4-52.

    The reference pulls `VivitConfig.from_pretrained(model_name)` and pretrained weights
    from the HF hub; this image has no network, so the architecture of the named
    checkpoint (ViViT-B/16x2) is built with seeded synthetic weights (vclip_amd.weights)
    unless a checkpoint is loaded afterwards with `load_state_dict`.  As in the
    reference, `num_labels` follows `class_labels` (id2label) and `num_frames` is set.
    """
    class_labels = class_labels or ["non-referral", "referral"]
    id2label = {i: l for i, l in enumerate(class_labels)}
    cfg = VivitConfig(num_frames=num_frames, id2label=id2label, label2id={l: i for i, l in id2label.items()})
    if logger:
        logger.info(f"Creating ViViT model {model_name} (num_frames={num_frames}, labels={class_labels}) on {device}")
    model = VivitForVideoClassification(cfg)
    from .weights import make_vivit_weights
    model.load_state_dict(make_vivit_weights(cfg.as_shape_cfg(), seed=weights_seed))
    model = model.to(device) if device else model
    return model.eval()  # like transformers' from_pretrained; the trainer calls model.train()
