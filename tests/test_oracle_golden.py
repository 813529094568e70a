"""Pin the oracle (oracle/vivit_ref.py) to goldens produced by HF transformers itself."""
import json
import os

import numpy as np
import torch

from oracle.vivit_ref import vivit_forward
from vclip_amd.weights import make_vivit_weights, make_synthetic_clips, sha256_state

GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_oracle_tiny_hidden_states():
    g = np.load(os.path.join(GD, "vivit_tiny.npz"))
    cfg = json.loads(str(g["config"]))
    sd = make_vivit_weights(cfg, seed=0)
    assert sha256_state(sd) == str(g["weights_sha256"])
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    logits, hid = vivit_forward(sdt, cfg, torch.from_numpy(g["pixel_values"]), return_hidden=True)
    np.testing.assert_allclose(hid.numpy(), g["hidden_states"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(logits.numpy(), g["logits"], rtol=0, atol=1e-5)


def test_oracle_full_vivit_b_logits():
    """ViViT-B/16x2 32f, B=2 (about 5 s on 8 cores)."""
    with open(os.path.join(GD, "vivit_full.json")) as f:
        g = json.load(f)
    cfg = g["config"]
    sd = make_vivit_weights(cfg, seed=g["weights_seed"])
    assert sha256_state(sd) == g["weights_sha256"]
    pix = make_synthetic_clips(g["batch"], cfg["num_frames"], cfg["image_size"], seed=g["input_seed"])
    import hashlib
    assert hashlib.sha256(pix.tobytes()).hexdigest() == g["pixel_sha256"]
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    with torch.no_grad():
        logits = vivit_forward(sdt, cfg, torch.from_numpy(pix))
    np.testing.assert_allclose(logits.numpy(), np.array(g["logits"]), rtol=0, atol=1e-5)


def test_oracle_timesformer_tiny_hidden_states():
    from oracle.timesformer_ref import timesformer_forward
    from vclip_amd.weights import make_timesformer_weights
    g = np.load(os.path.join(GD, "timesformer_tiny.npz"))
    cfg = json.loads(str(g["config"]))
    sd = make_timesformer_weights(cfg, seed=0)
    assert sha256_state(sd) == str(g["weights_sha256"])
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    logits, hid = timesformer_forward(sdt, cfg, torch.from_numpy(g["pixel_values"]), return_hidden=True)
    np.testing.assert_allclose(hid.numpy(), g["hidden_states"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(logits.numpy(), g["logits"], rtol=0, atol=1e-5)


def test_oracle_full_timesformer_b_logits():
    """TimeSformer-B 8f, B=2."""
    import hashlib
    from oracle.timesformer_ref import timesformer_forward
    from vclip_amd.weights import make_timesformer_weights
    with open(os.path.join(GD, "timesformer_full.json")) as f:
        g = json.load(f)
    cfg = g["config"]
    sd = make_timesformer_weights(cfg, seed=g["weights_seed"])
    assert sha256_state(sd) == g["weights_sha256"]
    pix = make_synthetic_clips(g["batch"], cfg["num_frames"], cfg["image_size"], seed=g["input_seed"])
    assert hashlib.sha256(pix.tobytes()).hexdigest() == g["pixel_sha256"]
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    with torch.no_grad():
        logits = timesformer_forward(sdt, cfg, torch.from_numpy(pix))
    np.testing.assert_allclose(logits.numpy(), np.array(g["logits"]), rtol=0, atol=1e-5)
