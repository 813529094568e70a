"""Fused AdamW on libvclip.so — drop-in for the reference's
`torch.optim.AdamW(model.parameters(), lr=args.learning_rate, weight_decay=args.weight_decay)`
(vivit_transformer/main.py:150-155), stepped at trainers/trainer.py:146.

Same constructor, same update (decoupled weight decay, bias-corrected moments, torch's
arithmetic order: vc_adamw).  When the parameters are the flat-buffer views of a
`vclip_amd.vivit.VivitForVideoClassification` in training (and their gradients the matching
views of its flat gradient buffer), the whole model is updated by ONE kernel launch over the
flat buffers (88.6M fp32 parameters at ViViT-B: an HBM-bound pass of 16 B read + 12 B
written per parameter).  Any other parameter list is updated tensor by tensor with the same
kernel.  `grad_scale` multiplies gradients first (1/world_size when they were SUM-reduced).
"""
from __future__ import annotations

import torch

from . import ops
from . import vivit_train


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.grad_scale = grad_scale
        self._flat_state = None  # (param storage ptr, grad storage ptr, exp_avg, exp_avg_sq, step)
        # device-step mode (vclip_amd.vivit_train.GraphedTrainStep): the flat update reads its step from a
        # device counter and bias-correction table, so a captured step stays correct on every replay
        self._dev_step = None  # (tab f32 [steps, 2], counter int64 [1])

    @staticmethod
    def _flat_view_set(params):
        """(param base tensor, grad base tensor) if every param / grad is a view of one flat
        buffer at matching offsets (the ViViT training layout), else None."""
        if not params or any(p.grad is None for p in params):
            return None
        ps = {p.untyped_storage().data_ptr() for p in params}
        gs = {p.grad.untyped_storage().data_ptr() for p in params}
        if len(ps) != 1 or len(gs) != 1:
            return None
        for p in params:
            if (p.dtype != torch.float32 or p.grad.dtype != torch.float32 or p.storage_offset() != p.grad.storage_offset()
                    or not p.is_contiguous() or not p.grad.is_contiguous() or p.device.type != "cuda"):
                return None
        p0, g0 = params[0], params[0].grad
        n = p0.untyped_storage().nbytes() // 4
        if g0.untyped_storage().nbytes() // 4 != n:
            return None
        # the single launch updates the WHOLE flat buffer: only when the parameters cover it
        # exactly, or are every entry of a ViViT flat layout (whose alignment gaps are zero in
        # both buffers, which AdamW leaves at zero); a subset, e.g. fine-tuning the head only,
        # goes tensor by tensor
        offs = {p.storage_offset() for p in params}
        if len(offs) != len(params):
            return None
        tags = {getattr(p, "_vc_flat_layout", None) for p in params}
        full_layout = len(tags) == 1 and None not in tags and tags == {(n, len(params))}
        if not full_layout and sum(p.numel() for p in params) != n:
            return None
        flat_p = torch.empty(0, dtype=torch.float32, device=p0.device).set_(p0.untyped_storage(), 0, (n,))
        flat_g = torch.empty(0, dtype=torch.float32, device=p0.device).set_(g0.untyped_storage(), 0, (n,))
        return flat_p, flat_g

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            params = [p for p in group["params"] if p.grad is not None]
            flat = self._flat_view_set(params) if len(self.param_groups) == 1 else None
            if flat is not None:
                fp, fg = flat
                # keyed by the layout (size, parameter count), not by device pointers, so the moments
                # survive a state_dict round trip or a re-flattened model of the same layout
                key = (fp.numel(), len(params))
                st = self.state.setdefault("flat", {})
                if st.get("key") != key:
                    st.update(key=key, exp_avg=torch.zeros_like(fp), exp_avg_sq=torch.zeros_like(fp), step=0)
                st["step"] += 1
                if self._dev_step is not None:
                    tab, counter = self._dev_step
                    ops.adamw_tab(fp, fg, st["exp_avg"], st["exp_avg_sq"], lr, b1, b2, eps, wd, tab, counter,
                                  self.grad_scale)
                    ops.adamw_step_tick(counter)
                else:
                    ops.adamw(fp, fg, st["exp_avg"], st["exp_avg_sq"], lr, b1, b2, eps, wd, st["step"],
                              self.grad_scale)
            else:
                if self._dev_step is not None:
                    raise RuntimeError("AdamW device-step mode (a captured train step) needs the model's flat buffers")
                # every tensor of the group in one multi-tensor launch per distinct step count
                by_step = {}
                for p in params:
                    st = self.state[p]
                    if not st:
                        st.update(exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p), step=0)
                    st["step"] += 1
                    g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                    by_step.setdefault(st["step"], []).append((p, g, st["exp_avg"], st["exp_avg_sq"]))
                for step, quads in by_step.items():
                    if len(quads) == 1 or not all(q.is_contiguous() for q, _, _, _ in quads):
                        for p, g, m, v in quads:
                            ops.adamw(p, g, m, v, lr, b1, b2, eps, wd, step, self.grad_scale)
                    else:
                        self._tables = ops.adamw_multi(*zip(*quads), lr, b1, b2, eps, wd, step, self.grad_scale)
        vivit_train.MASTER_EPOCH[0] += 1
        return loss
