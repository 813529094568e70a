"""Checkpoint key compatibility.

The reference saves `model.state_dict()` of a transformers-4.48.2 model inside a dict
(vivit_transformer/vivit_classifier/trainers/trainer.py:291-305: epoch,
model_state_dict, optimizer_state_dict, ..., config, id2label, label2id) and reloads it
in inference (vivit_transformer/inference.py:37-69); DataParallel checkpoints carry a
`module.` prefix (stripped as in videoswintransformer/inference.py:73-87).  Keys are
renamed to the transformers-5 names this package uses, following the published rename
rules (TF5/conversion_mapping.py:338-346).
"""
from __future__ import annotations

import re
from collections import OrderedDict

_RULES = [
    (r"^module\.", ""),
    (r"encoder\.layer\.", "layers."),
    (r"attention\.attention\.query", "attention.q_proj"),
    (r"attention\.attention\.key", "attention.k_proj"),
    (r"attention\.attention\.value", "attention.v_proj"),
    (r"attention\.output\.dense", "attention.o_proj"),
    (r"intermediate\.dense", "mlp.fc1"),
    (r"\.output\.dense", ".mlp.fc2"),
]


def convert_key(k: str) -> str:
    for pat, rep in _RULES:
        k = re.sub(pat, rep, k)
    return k


def convert_state_dict(sd) -> "OrderedDict":
    return OrderedDict((convert_key(k), v) for k, v in sd.items())


def load_reference_checkpoint(path: str, map_location="cpu", vivit_keys: bool = True):
    """Load a reference `.pth` training checkpoint dict safely (weights_only=True).  vivit_keys:
    rename transformers-4.48 ViViT keys (the other families' models strip `module.` themselves)."""
    import torch
    ck = torch.load(path, map_location=map_location, weights_only=True)
    conv = convert_state_dict if vivit_keys else (lambda sd: OrderedDict(sd))
    if isinstance(ck, dict) and "model_state_dict" in ck:
        return ck, conv(ck["model_state_dict"])
    return {}, conv(ck)
