"""ViViT train step on libvclip.so: forward with saved activations, backward, gradients in
one flat fp32 buffer.

Reference step (vivit_transformer/vivit_classifier/trainers/trainer.py:140-146):
    optimizer.zero_grad(); outputs = model(**inputs); loss = criterion(outputs.logits, labels)
    loss.backward(); optimizer.step()
with criterion = nn.CrossEntropyLoss() and AdamW(lr, weight_decay) (vivit_transformer/main.py:150-155).
That exact loop runs unchanged on `vclip_amd.vivit.VivitForVideoClassification`: in train mode
with grad enabled, the model's forward goes through `VivitTrainFn`, an autograd.Function whose
backward runs the HIP backward kernels and writes every parameter's gradient into the flat
gradient buffer (`p.grad` are views of it).  The loss itself stays torch's CrossEntropyLoss on
the [B, 2] logits; its dlogits enter the kernels' head backward.

Flat layout (fp32 masters and gradients share it; each tensor 64-element aligned).  The order
is the order in which the backward finishes gradients — classifier, final LayerNorm, layers
L-1 .. 0, embeddings — so finished gradients always form a growing prefix and a data-parallel
all-reduce can start on each layer's slice while the layers below are still in the backward
(`grad_ready_hooks`).  Within a layer q|k|v weights and biases are adjacent, so the fused
[3D, D] projection and its gradient are plain views.
"""
from __future__ import annotations

import math

import torch

from . import ops, streams

ALIGN = 64

# bumped by vclip_amd.optim.AdamW after it rewrites fp32 masters through raw pointers (no torch
# version-counter bump), so inference-side bf16 packs know to refresh
MASTER_EPOCH = [0]


def _round_up(x, m):
    return (x + m - 1) // m * m


def flat_order(cfg) -> list:
    """HF parameter names in flat-buffer order (the backward's gradient-completion order)."""
    L = cfg.num_hidden_layers
    names = ["classifier.weight", "classifier.bias", "vivit.layernorm.weight", "vivit.layernorm.bias"]
    for i in reversed(range(L)):
        p = f"vivit.layers.{i}."
        names += [p + "attention.q_proj.weight", p + "attention.k_proj.weight", p + "attention.v_proj.weight",
                  p + "attention.q_proj.bias", p + "attention.k_proj.bias", p + "attention.v_proj.bias",
                  p + "attention.o_proj.weight", p + "attention.o_proj.bias",
                  p + "layernorm_before.weight", p + "layernorm_before.bias",
                  p + "layernorm_after.weight", p + "layernorm_after.bias",
                  p + "mlp.fc1.weight", p + "mlp.fc1.bias", p + "mlp.fc2.weight", p + "mlp.fc2.bias"]
    names += ["vivit.embeddings.patch_embeddings.projection.weight", "vivit.embeddings.patch_embeddings.projection.bias",
              "vivit.embeddings.cls_token", "vivit.embeddings.position_embeddings"]
    return names


class FlatLayout:
    """name -> (offset, numel, shape) in the flat buffer; q|k|v weights / biases are placed
    back to back (no alignment gap) so they form one [3D, D] / [3D] tensor."""

    def __init__(self, cfg, shapes: dict):
        self.entries = {}
        off = 0
        order = flat_order(cfg)
        assert sorted(order) == sorted(shapes), "flat_order must cover every parameter exactly once"
        for n in order:
            shp = tuple(shapes[n])
            numel = math.prod(shp)
            tight = n.endswith(("k_proj.weight", "v_proj.weight", "k_proj.bias", "v_proj.bias"))
            if not tight:
                off = _round_up(off, ALIGN)
            self.entries[n] = (off, numel, shp)
            off += numel
        self.total = _round_up(off, ALIGN)
        # slices whose gradients complete together, in completion order
        L = cfg.num_hidden_layers
        first = lambda i: self.entries[f"vivit.layers.{i}.attention.q_proj.weight"][0]  # noqa: E731
        emb0 = self.entries["vivit.embeddings.patch_embeddings.projection.weight"][0]
        self.stages = [("head", 0, first(L - 1))]
        for i in reversed(range(L)):
            self.stages.append((f"layer{i}", first(i), first(i - 1) if i > 0 else emb0))
        self.stages.append(("embeddings", emb0, self.total))

    def view(self, flat: torch.Tensor, name: str, shape=None) -> torch.Tensor:
        off, numel, shp = self.entries[name]
        return flat[off:off + numel].view(shape if shape is not None else shp)

    def span(self, flat: torch.Tensor, first: str, count: int, shape) -> torch.Tensor:
        """`count` elements starting at `first` (the q|k|v block), viewed as `shape`."""
        off = self.entries[first][0]
        return flat[off:off + count].view(shape)


class TrainEngine:
    """Device buffers and the kernel sequence of one training step for a fixed batch size."""

    def __init__(self, model, B: int, device):
        c = model.config
        self.model, self.B, self.device = model, B, device
        D, I, H = c.hidden_size, c.intermediate_size, c.num_attention_heads
        kt, kh, kw = c.tubelet_size
        npatch, S, Mpad, Memb = model.geometry(B)
        self.D, self.I, self.H, self.S, self.Mpad, self.Memb, self.npatch = D, I, H, S, Mpad, Memb, npatch
        self.Kemb = c.num_channels * kt * kh * kw
        L = c.num_hidden_layers
        self.L = L
        bf, f32 = torch.bfloat16, torch.float32
        z = lambda *s, dt=bf: torch.zeros(s, dtype=dt, device=device)  # noqa: E731
        # saved forward activations
        self.A_emb = z(Memb, self.Kemb)
        self.R = [z(Mpad, D, dt=f32) for _ in range(2 * L + 1)]  # residual stream before/after each block
        self.Y1 = [z(Mpad, D) for _ in range(L)]
        self.QKV = [z(Mpad, 3 * D) for _ in range(L)]
        self.O = [z(Mpad, D) for _ in range(L)]
        self.LSE = [z(B * H * S, dt=f32) for _ in range(L)]
        self.Y2 = [z(Mpad, D) for _ in range(L)]
        self.Hpre = [z(Mpad, I) for _ in range(L)]
        self.Hd = [z(Mpad, I) for _ in range(L)]
        self.logits = z(B, c.num_labels, dt=f32)
        # backward scratch
        self.dX = z(Mpad, D, dt=f32)
        self.dXb = z(Mpad, D)    # bf16 gradient at a block's input (head / layernorm_before backward)
        self.dXb2 = z(Mpad, D)   # bf16 gradient between the attention and MLP blocks (layernorm_after backward)
        self.dY = z(Mpad, D, dt=f32)
        self.dH = z(Mpad, I)
        self.dO = z(Mpad, D)
        self.dQKV = z(Mpad, 3 * D)
        self.delta = z(B * H * S, dt=f32)
        self.demb = z(Memb, D)
        self.work = z(max(16 * max(I, 3 * D) * D, (512 + 16) * 2 * D, 256 * max(I, 3 * D)), dt=f32)
        # weight / bias gradients on a side stream, beside the data-gradient chain (split-K tails, the
        # partial reductions and the column sums fill what the dgrad GEMMs and the attention backward
        # leave idle); its own split-K scratch.  False: everything on the caller's stream.
        self.side_wgrad = True
        self.side = None
        self.work_side = torch.zeros_like(self.work)
        # cap on the split-K factor of the weight gradients (None: vc_wgrad_bf16's own ~one-workgroup-
        # per-CU choice, 10 - 28 partials here); the scratch handed over bounds the splits.  Beside the
        # data-gradient chain fewer, longer workgroups win: 4 -> 214.3 clips/s vs 205.7 uncapped, 208.1
        # at 8, 206.4 at 2 (tools/ab_train_side.py, one process, round 4)
        self.wgrad_max_splits = 4
        # the attention backward's dQ kernel on a stream of its own beside dK/dV (vc_attention_bwd_2s)
        self.attn_bwd_2s = True
        self.side_dq = None
        # tile-configuration overrides of the backward's data-gradient GEMMs (vc_gemm_bf16_cfg; name ->
        # cfg): "dgelu" (fc2^T with the gelu' epilogue), "dfc1" (fc1^T), "do" (o_proj^T), "dqkv" (q|k|v^T)
        self.gemm_cfg = {}
        self.zeros = z(max(I, 3 * D, self.Kemb), dt=f32)
        # packed bf16 weights (forward operand W [N, K] and dgrad operand W^T [K, N]) + packed q|k|v bias
        self.W = [dict(qkv=z(3 * D, D), qkvT=z(D, 3 * D), o=z(D, D), oT=z(D, D), f1=z(I, D), f1T=z(D, I),
                       f2=z(D, I), f2T=z(I, D), bqkv=z(3 * D, dt=f32)) for _ in range(L)]
        self.W_emb = z(D, self.Kemb)
        self.kernel_events = None

    # ---- weights ------------------------------------------------------------------------------
    def pack(self):
        """fp32 masters -> bf16 operands (every step: the optimizer moved the masters)."""
        lay, flat = self.model._layout, self.model._flat
        D = self.D
        qs = (D // self.H) ** -0.5 * ops.LOG2E
        ops.pack_weight(lay.view(flat, "vivit.embeddings.patch_embeddings.projection.weight", (D, self.Kemb)),
                        dst=self.W_emb)
        for i, W in enumerate(self.W):
            p = f"vivit.layers.{i}."
            wqkv = lay.span(flat, p + "attention.q_proj.weight", 3 * D * D, (3 * D, D))
            ops.pack_weight(wqkv, W["qkv"], W["qkvT"], nscaled=D, scale=qs)
            ops.pack_weight(lay.view(flat, p + "attention.o_proj.weight"), W["o"], W["oT"])
            ops.pack_weight(lay.view(flat, p + "mlp.fc1.weight"), W["f1"], W["f1T"])
            ops.pack_weight(lay.view(flat, p + "mlp.fc2.weight"), W["f2"], W["f2T"])
            bqkv = lay.span(flat, p + "attention.q_proj.bias", 3 * D, (3 * D,))
            torch.mul(bqkv[:D], qs, out=W["bqkv"][:D])
            W["bqkv"][D:].copy_(bqkv[D:])

    # ---- forward ------------------------------------------------------------------------------
    def forward(self, pix: torch.Tensor) -> torch.Tensor:
        m, lay, flat = self.model, self.model._layout, self.model._flat
        c = m.config
        D, S, B, H = self.D, self.S, self.B, self.H
        eps = c.layer_norm_eps
        P = lambda n: lay.view(flat, n)  # noqa: E731
        self.pack()
        ops.tubelet_im2col(pix, c.tubelet_size, self.A_emb)
        pos = P("vivit.embeddings.position_embeddings").view(S, D)
        ops.gemm(self.A_emb, self.W_emb, P("vivit.embeddings.patch_embeddings.projection.bias"), "embed_f32", self.R[0],
                 aux=pos[1:], group=self.npatch, group_stride=S, group_offset=1, m=self.Memb)
        ops.cls_init(P("vivit.embeddings.cls_token").view(D), pos, self.R[0], B, S)
        for i in range(self.L):
            p = f"vivit.layers.{i}."
            W = self.W[i]
            ops.layernorm(self.R[2 * i], P(p + "layernorm_before.weight"), P(p + "layernorm_before.bias"), eps, self.Y1[i])
            ops.gemm(self.Y1[i], W["qkv"], W["bqkv"], "bias", self.QKV[i])
            ops.attention_fwd_lse(self.QKV[i], B, S, H, self.O[i], self.LSE[i])
            ops.gemm(self.O[i], W["o"], P(p + "attention.o_proj.bias"), "bias_add_f32", self.R[2 * i + 1],
                     aux=self.R[2 * i])
            ops.layernorm(self.R[2 * i + 1], P(p + "layernorm_after.weight"), P(p + "layernorm_after.bias"), eps,
                          self.Y2[i])
            ops.gemm(self.Y2[i], W["f1"], P(p + "mlp.fc1.bias"), "bias_gelu_tanh_save", self.Hd[i], aux=self.Hpre[i])
            ops.gemm(self.Hd[i], W["f2"], P(p + "mlp.fc2.bias"), "bias_add_f32", self.R[2 * i + 2],
                     aux=self.R[2 * i + 1])
        return ops.cls_head(self.R[2 * self.L], B, S, P("vivit.layernorm.weight"), P("vivit.layernorm.bias"), eps,
                            P("classifier.weight"), P("classifier.bias"), out=self.logits)

    # ---- backward -----------------------------------------------------------------------------
    def backward(self, dlogits: torch.Tensor, gflat: torch.Tensor, ready=None):
        """Gradients of every parameter into gflat (overwritten); `ready(stage, start, end)` is
        called as each stage's slice of gflat is complete (enqueued on the current stream)."""
        m, lay, flat = self.model, self.model._layout, self.model._flat
        c = m.config
        D, I, S, B, H = self.D, self.I, self.S, self.B, self.H
        eps = c.layer_norm_eps
        qs = (D // H) ** -0.5 * ops.LOG2E
        P = lambda n: lay.view(flat, n)  # noqa: E731
        G = lambda n, shape=None: lay.view(gflat, n, shape)  # noqa: E731
        ready = ready or (lambda *a: None)
        stages = {s[0]: s for s in lay.stages}
        dX, dXa, dXb, dY, dH, dO, dQKV = self.dX, self.dXb, self.dXb2, self.dY, self.dH, self.dO, self.dQKV
        main = torch.cuda.current_stream(self.device)
        side_on = self.side_wgrad
        if side_on and self.side is None:
            # the weight-gradient, dQ and gradient all-reduce side streams, measured to run beside each
            # other and beside the main stream (streams.pick_streams): streams drawn blind ran the step
            # at 183 / 206 instead of 220 clips/s in 5 of 12 trials (tools/exp_train_streams.py)
            self.side = streams.pick_streams(self.device, 3, against=(main,))[0]
        ws0 = self.work_side if side_on else self.work

        class _WS:  # the split-K scratch of one weight gradient, capped at wgrad_max_splits partials
            def __init__(s2, cap):
                s2.cap = cap  # int, or {"fc2" | "fc1" | "o" | "qkv": int} (absent: 4)

            def __call__(s2, out, name):
                cap = s2.cap.get(name, 4) if isinstance(s2.cap, dict) else s2.cap
                if cap is None:
                    return ws0
                return ws0[: min(ws0.numel(), max(2, cap) * out.numel())]

        wsf = _WS(self.wgrad_max_splits)
        ws = ws0

        def on_side(fn):
            """fn() (weight / bias gradients whose operands main has produced by now) on the side
            stream; returns the event main waits on before it overwrites those operands"""
            if not side_on:
                fn()
                return None
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                fn()
            e = torch.cuda.Event()
            e.record(self.side)
            return e

        def wait(e):
            if e is not None:
                main.wait_event(e)

        gc = lambda name: self.gemm_cfg.get(name, -1)  # noqa: E731

        dX.zero_()
        dXa.zero_()
        ops.cls_head_bwd(self.R[2 * self.L], B, S, P("vivit.layernorm.weight"), P("vivit.layernorm.bias"), eps,
                         P("classifier.weight"), dlogits, dX, dXa, G("classifier.weight"), G("classifier.bias"),
                         G("vivit.layernorm.weight"), G("vivit.layernorm.bias"))
        ready(*stages["head"])
        ev_fc1 = ev_o = ev_qkv = None  # the previous (deeper) layer's side work on dH / dXb / dQKV
        pending = None                 # (side event, stage) of a layer whose gradients are complete there
        for i in reversed(range(self.L)):
            p = f"vivit.layers.{i}."
            W = self.W[i]
            # MLP block: out = R1 + fc2(gelu(fc1(LN2(R1))))
            wait(ev_fc1)  # dH was read by the previous layer's fc1 weight / bias gradients
            ops.gemm(dXa, W["f2T"], self.zeros[:I], "dgelu_tanh", dH, aux=self.Hpre[i], cfg=gc("dgelu"))
            ev_fc2 = on_side(lambda: ops.wgrad(dXa, self.Hd[i], G(p + "mlp.fc2.weight"), wsf(G(p + "mlp.fc2.weight"), "fc2")))
            ops.gemm(dH, W["f1T"], self.zeros[:D], "bias_f32", dY, cfg=gc("dfc1"))
            ev_fc1 = on_side(lambda: (ops.wgrad(dH, self.Y2[i], G(p + "mlp.fc1.weight"), wsf(G(p + "mlp.fc1.weight"), "fc1")),
                                      ops.colsum(dH, G(p + "mlp.fc1.bias"), ws)))
            # + the fc2 / o_proj bias gradients: column sums of dX before / after this update
            wait(ev_o)  # dXb was read by the previous layer's o_proj weight gradient
            ops.layernorm_bwd(dY, self.R[2 * i + 1], P(p + "layernorm_after.weight"), eps, dX, dXb,
                              G(p + "layernorm_after.weight"), G(p + "layernorm_after.bias"), self.work, m=B * S,
                              dsum_in=G(p + "mlp.fc2.bias"), dsum_out=G(p + "attention.o_proj.bias"))
            # attention block: R1 = R0 + o_proj(attn(qkv(LN1(R0))))
            ops.gemm(dXb, W["oT"], self.zeros[:D], "bias", dO, cfg=gc("do"))
            ev_o = on_side(lambda: ops.wgrad(dXb, self.O[i], G(p + "attention.o_proj.weight"), wsf(G(p + "attention.o_proj.weight"), "o")))
            wait(ev_qkv)  # dQKV was read by the previous layer's q|k|v weight / bias gradients
            ev = self.kernel_events  # optional HIP-event timing of the attention backward (bench.py)
            if ev is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            if self.attn_bwd_2s and self.side_dq is None:
                self.side_dq = streams.pick_streams(self.device, 3, against=(main,))[1]
            ops.attention_bwd(self.QKV[i], self.O[i], dO, self.LSE[i], self.delta, B, S, H, dQKV,
                              stream2=self.side_dq if self.attn_bwd_2s else None)
            if ev is not None:
                e1.record()
                ev.append((e0, e1))
            ops.gemm(dQKV, W["qkvT"], self.zeros[:D], "bias_f32", dY, cfg=gc("dqkv"))
            ev_qkv = on_side(lambda: (
                ops.wgrad(dQKV, self.Y1[i], lay.span(gflat, p + "attention.q_proj.weight", 3 * D * D, (3 * D, D)),
                          wsf(lay.span(gflat, p + "attention.q_proj.weight", 3 * D * D, (3 * D, D)), "qkv"), nscaled=D,
                          scale=qs),
                ops.colsum(dQKV, lay.span(gflat, p + "attention.q_proj.bias", 3 * D, (3 * D,)), ws,
                           nscaled=D, scale=qs)))
            wait(ev_fc2)  # dXa was read by this layer's fc2 weight gradient
            ops.layernorm_bwd(dY, self.R[2 * i], P(p + "layernorm_before.weight"), eps, dX, dXa,
                              G(p + "layernorm_before.weight"), G(p + "layernorm_before.bias"), self.work, m=B * S)
            # a layer's gradients are announced one layer later, when its side work has long finished
            if pending is not None:
                wait(pending[0])
                ready(*pending[1])
            pending = (ev_qkv, stages[f"layer{i}"])
        if pending is not None:
            wait(pending[0])
            ready(*pending[1])
        if side_on:
            main.wait_stream(self.side)
        gpos = G("vivit.embeddings.position_embeddings").view(S, D)
        ops.embed_bwd(dX, B, S, gpos, G("vivit.embeddings.cls_token").view(D), self.demb)
        ops.wgrad(self.demb, self.A_emb, G("vivit.embeddings.patch_embeddings.projection.weight", (D, self.Kemb)),
                  self.work)
        ops.colsum(gpos[1:], G("vivit.embeddings.patch_embeddings.projection.bias"), self.work)
        ready(*stages["embeddings"])


class VivitTrainFn(torch.autograd.Function):
    """logits = ViViT(pixel_values) with the HIP forward; backward = the HIP backward, which
    writes the parameter gradients into the model's flat gradient buffer itself (p.grad are
    views of it) and returns None for every input."""

    @staticmethod
    def forward(ctx, model, pix, *params):
        eng = model._train_engine(pix.shape[0], pix.device)
        logits = eng.forward(pix)
        ctx.model, ctx.engine = model, eng
        return logits.clone()

    @staticmethod
    def backward(ctx, dlogits):
        model, eng = ctx.model, ctx.engine
        model._run_backward(eng, dlogits.float().contiguous())
        return (None, None) + (None,) * len(model._param_list())


class GraphedTrainStep:
    """The reference's train step (vivit_transformer/vivit_classifier/trainers/trainer.py:140-146:
    zero_grad, model(**inputs), CrossEntropyLoss, backward, optimizer.step) captured once into a hipGraph and
    replayed: ~450 HIP launches per ViViT-B step over three streams (the data-gradient chain, the weight
    gradients beside it, the attention backward's dQ) go to the GPU as one graph, with no host launch work
    per step.  The same kernels in the same order as the eager step, so parameters, moments and losses are
    bit-identical to it (tests/test_vivit_train_gpu.py).  At ViViT-B B = 4 the eager step is not
    launch-bound and the replay measured 2 % slower (212.3 vs 216.6 clips/s, round 6), so bench.py runs it
    only with --train-graph 1; it is for steps whose launches the host cannot keep ahead of.

        step = GraphedTrainStep(model, optimizer, criterion, pixel_values, labels)
        loss = step(pixel_values, labels)   # new inputs are copied into the captured buffers

    Needs the flat-buffer AdamW of vclip_amd.optim (its step count moves to a device counter, so the
    captured update stays correct on every replay) and no grad_ready_hooks (the data-parallel all-reduce
    runs eagerly; bench.py captures at world size 1 only).  Capture happens after `warmup` eager steps
    (workspaces, packs, kernel attributes are created outside the capture).  Host-side state that the eager
    step advances (the optimizer's step count, MASTER_EPOCH for the inference packs) is advanced per replay."""

    MAX_STEPS = 1 << 20  # rows of the device bias-correction table (8 MiB)

    def __init__(self, model, optimizer, criterion, pixel_values, labels, warmup: int = 2):
        from .optim import AdamW
        if not isinstance(optimizer, AdamW):
            raise TypeError("GraphedTrainStep needs vclip_amd.optim.AdamW")
        if model.grad_ready_hooks:
            raise RuntimeError("GraphedTrainStep: grad_ready_hooks (data-parallel all-reduce) run eagerly")
        if len(optimizer.param_groups) != 1:
            raise RuntimeError("GraphedTrainStep: one parameter group (the flat-buffer update)")
        self.model, self.opt, self.crit = model, optimizer, criterion
        dev = pixel_values.device
        self.pix = pixel_values.detach().clone()
        self.labels = labels.detach().clone()

        def eager():
            self.opt.zero_grad()
            out = self.model(pixel_values=self.pix)
            loss = self.crit(out.logits, self.labels)
            loss.backward()
            self.opt.step()
            return loss

        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                eager()
        torch.cuda.current_stream(dev).wait_stream(side)
        st = self.opt.state.get("flat")
        if st is None:
            raise RuntimeError("GraphedTrainStep: the optimizer did not take the flat-buffer path")
        g = self.opt.param_groups[0]
        b1, b2 = g["betas"]
        self.tab = ops.adamw_step_table(b1, b2, g["lr"], self.MAX_STEPS, dev)
        self.counter = torch.tensor([st["step"]], dtype=torch.int64, device=dev)
        self._hyper = (g["lr"], b1, b2, g["eps"], g["weight_decay"], self.opt.grad_scale)
        self.opt.zero_grad()
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        self.opt._dev_step = (self.tab, self.counter)
        try:
            with torch.cuda.graph(self.graph):
                out = self.model(pixel_values=self.pix)
                self.loss = self.crit(out.logits, self.labels)
                self.loss.backward()
                self.opt.step()
        finally:
            self.opt._dev_step = None
        st["step"] -= 1  # the capture ran the step's host code once without running the step
        MASTER_EPOCH[0] -= 1

    def __call__(self, pixel_values=None, labels=None) -> torch.Tensor:
        g = self.opt.param_groups[0]
        if (g["lr"], *g["betas"], g["eps"], g["weight_decay"], self.opt.grad_scale) != self._hyper:
            raise RuntimeError("GraphedTrainStep: optimizer hyper-parameters changed since the capture; build a new step")
        st = self.opt.state["flat"]
        if st["step"] >= self.MAX_STEPS:
            raise RuntimeError("GraphedTrainStep: past the bias-correction table; build a new step")
        if pixel_values is not None and pixel_values.data_ptr() != self.pix.data_ptr():
            self.pix.copy_(pixel_values)
        if labels is not None and labels.data_ptr() != self.labels.data_ptr():
            self.labels.copy_(labels)
        self.graph.replay()
        st["step"] += 1
        MASTER_EPOCH[0] += 1
        return self.loss
