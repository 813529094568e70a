"""Generate the committed golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the survey/build container (needs /root/reference and HF transformers);
never on the GPU box.  The reference code is imported read-only (bytecode writing is
disabled so nothing lands in /root/reference) with its absent third-party imports
(cv2, av, pytorchvideo, torchvision, matplotlib, ...) replaced by inert stub modules:
the sampling functions only touch Python `random`, `numpy.random` and, on the
short-video branch, `cv2.VideoCapture(path).get(CAP_PROP_FPS)`.

Outputs (all data, no reference source):
  tests/golden/sampling.json     sampled frame indices for every sampler variant
  tests/golden/vivit_tiny.npz    tiny ViViT: inputs, weights seed, logits + hidden states
  tests/golden/vivit_full.json   ViViT-B/16x2 32f logits (B=2) + sha256 of weights/inputs
  tests/golden/timesformer_tiny.npz / timesformer_full.json   the same for TimeSformer (8f)
  tests/golden/timesformer_tiny.npz  tiny TimeSformer logits (for the next §8 row)

Usage:  PYTHONDONTWRITEBYTECODE=1 PYTHONHASHSEED=0 python tools/make_goldens.py [--skip-full]
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import importlib.abc
import importlib.util
import json
import os
import sys
import types
from types import SimpleNamespace

sys.dont_write_bytecode = True
REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

# --------------------------------------------------------------------------- stubs
_FPS_BY_PATH: dict[str, float] = {}


class _Anything:
    """Inert stand-in: callable, attribute-able, subclassable."""

    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Anything()

    def __getattr__(self, name):
        return _Anything()


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Anything


class _Cap:
    def __init__(self, path):
        self.path = str(path)

    def get(self, prop):
        return _FPS_BY_PATH.get(self.path, 30.0)

    def release(self):
        pass

    def isOpened(self):
        return True


_STUB_ROOTS = ("cv2", "av", "pytorchvideo", "torchvision", "matplotlib", "seaborn", "wandb")


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if fullname.split(".")[0] in _STUB_ROOTS:
            return importlib.util.spec_from_loader(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _StubModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


def _install_stubs():
    sys.meta_path.insert(0, _StubFinder())
    import cv2  # noqa: F401  (stub)
    cv2 = sys.modules["cv2"]
    cv2.VideoCapture = _Cap
    cv2.CAP_PROP_FPS = 5
    cv2.CAP_PROP_FRAME_COUNT = 7


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Log:
    def info(self, *a, **k):
        pass

    warning = debug = error = info


# --------------------------------------------------------------------------- sampling
TOTALS = [1, 7, 20, 31, 32, 33, 64, 300, 10007]
NUMS = [1, 8, 16, 32]
METHODS = ["uniform", "random_window", "random"]


def _sequences():
    """Call sequences (lists of (basename, total_frames)) replayed after construction."""
    seqs = []
    for t in TOTALS:
        seqs.append([(f"v{t:05d}.mp4", t)])
    seqs.append([("0047.mp4", 300), ("0012.mp4", 33), ("0047.mp4", 300), ("0101.mp4", 7),
                 ("0200.mp4", 10007), ("0012.mp4", 31), ("0300.mp4", 64), ("0301.mp4", 1)])
    return seqs


def gen_sampling():
    import random
    import numpy as np
    import torch  # noqa: F401  (resnet3d set_random_seed calls torch.manual_seed)

    _install_stubs()
    mods = {}
    mods["vivit"] = _load(f"{REF}/vivit_transformer/vivit_classifier/data_config/dataset.py", "ref_vivit_ds")
    mods["timesformer"] = _load(f"{REF}/timesformer/timesformer_classifier/data_config/dataset.py", "ref_tsf_ds")
    mods["swin"] = _load(f"{REF}/videoswintransformer/swin_video_classifier/data_config/dataset.py", "ref_swin_ds")
    mods["resnet3d"] = _load(f"{REF}/resnet50-3d-video/video_classifier/data_config/dataset.py", "ref_r3d_ds")
    mods["lstm"] = _load(f"{REF}/resnet50-2d-lstm/src/data_config/dataset.py", "ref_lstm_ds")
    sys.path.insert(0, f"{REF}/videoswintransformer")
    mods["swin_inf"] = _load(f"{REF}/videoswintransformer/inference.py", "ref_swin_inf")
    sys.path.pop(0)
    sys.path.insert(0, f"{REF}/resnet50-3d-video")
    mods["resnet3d_inf"] = _load(f"{REF}/resnet50-3d-video/inference.py", "ref_r3d_inf")
    sys.path.pop(0)
    sys.path.insert(0, f"{REF}/resnet50-2d-lstm")
    mods["lstm_inf"] = _load(f"{REF}/resnet50-2d-lstm/inference.py", "ref_lstm_inf")
    sys.path.pop(0)
    dh = _load(f"{REF}/data_handling.py", "ref_data_handling")

    # short videos take the fps branch for swin / resnet3d: give some paths odd fps values
    fps_table = {"v00007.mp4": 25.0, "v00020.mp4": 29.97, "v00031.mp4": 24.0, "0101.mp4": 12.5,
                 "0012.mp4": 30.0, "0301.mp4": 60.0, "v00001.mp4": 30.0}

    cases = []
    for variant in ["vivit", "timesformer", "swin", "swin_inf", "resnet3d", "resnet3d_inf", "lstm"]:
        for method in METHODS:
            for T in NUMS:
                for seq in _sequences():
                    _FPS_BY_PATH.clear()
                    for b, f in fps_table.items():
                        _FPS_BY_PATH[f"/data/{b}"] = f
                    # construction-time seeding (dataset __init__ reseeds 42, lstm does not)
                    random.seed(42)
                    np.random.seed(42)
                    if variant in ("vivit", "timesformer"):
                        ns = SimpleNamespace(num_frames=T, sampling_method=method, logger=_Log())
                        fn = lambda p, t, ns=ns, m=mods[variant]: m.VideoDataset.get_sampling_indices(ns, p, t)
                    elif variant == "swin":
                        ns = SimpleNamespace(num_frames=T, sampling_method=method, logger=_Log())
                        fn = lambda p, t, ns=ns, m=mods[variant]: list(m.VideoDataset.get_sampling_indices(ns, p, t))
                    elif variant == "swin_inf":
                        fn = lambda p, t, T=T, method=method, m=mods[variant]: list(
                            m.get_sampling_indices(p, t, T, method, _Log()))
                    elif variant == "resnet3d":
                        ns = SimpleNamespace(num_frames=T, sampling_method=method, logger=_Log(),
                                             cached_indices={}, fps=30)
                        ns.set_random_seed = lambda s, ns=ns, m=mods[variant]: m.VideoDataset.set_random_seed(ns, s)
                        fn = lambda p, t, ns=ns, m=mods[variant]: m.VideoDataset.get_sampling_indices(ns, p, t)
                    elif variant == "resnet3d_inf":
                        ns = SimpleNamespace(num_frames=T, sampling_method=method, logger=_Log(),
                                             sampled_frames={}, dynamic_fps_info={}, fps=30)
                        ns.set_random_seed = lambda s, ns=ns, m=mods[variant]: m.VideoInference.set_random_seed(ns, s)
                        fn = lambda p, t, ns=ns, m=mods[variant]: list(m.VideoInference.get_sampling_indices(ns, p, t))
                    elif variant == "lstm":
                        ns = SimpleNamespace(sequence_length=T, sampling_method=method, logger=_Log(), fps=30)
                        fn = lambda p, t, ns=ns, m=mods[variant]: m.VideoDataset.get_sampling_indices(ns, p, t)
                    calls = []
                    for base, total in seq:
                        out = fn(f"/data/{base}", total)
                        if variant in ("swin", "swin_inf", "resnet3d_inf"):
                            idx, dfps = out
                            calls.append({"path": f"/data/{base}", "total": total,
                                          "indices": [int(i) for i in idx],
                                          "dynamic_fps": None if dfps is None else float(dfps)})
                        else:
                            calls.append({"path": f"/data/{base}", "total": total,
                                          "indices": [int(i) for i in out]})
                    cases.append({"variant": variant, "method": method, "num_frames": T, "calls": calls})

    # resnet50-2d-lstm inference samplers (numpy RNG, num_frames clamped to total)
    lstm_inf = []
    for method, fname in [("random", "random_sampling"), ("uniform", "uniform_sampling"),
                          ("random_window", "random_window_sampling")]:
        for T in NUMS:
            for total in TOTALS:
                np.random.seed(42)
                f = getattr(mods["lstm_inf"].EnhancedVideoInference, fname)
                out = f(None, total, T)
                lstm_inf.append({"method": method, "num_frames": T, "total": total,
                                 "indices": [int(i) for i in out]})

    # data_handling.sample_frame_indices
    dh_cases = []
    for seed in [0, 42, 1234]:
        for clip_len, rate, seg_len in [(10, 1, 300), (32, 1, 300), (16, 4, 1000), (8, 2, 17), (32, 2, 65)]:
            np.random.seed(seed)
            seq = []
            for _ in range(3):
                seq.append([int(i) for i in dh.sample_frame_indices(clip_len, rate, seg_len)])
            dh_cases.append({"seed": seed, "clip_len": clip_len, "frame_sample_rate": rate,
                             "seg_len": seg_len, "calls": seq})

    out = {"generator": "tools/make_goldens.py", "PYTHONHASHSEED": os.environ.get("PYTHONHASHSEED"),
           "fps_table": fps_table, "cases": cases, "lstm_inference": lstm_inf,
           "sample_frame_indices": dh_cases}
    with open(os.path.join(GOLDEN, "sampling.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"sampling.json: {len(cases)} cases, {len(lstm_inf)} lstm-inference, {len(dh_cases)} data_handling")


# --------------------------------------------------------------------------- models
def _vivit_golden(cfg_kwargs, batch, wseed, xseed, full):
    import numpy as np
    import torch
    from transformers import VivitConfig, VivitForVideoClassification

    sys.path.insert(0, ROOT)
    from vclip_amd.weights import make_vivit_weights, make_synthetic_clips, sha256_state

    cfg = VivitConfig(**cfg_kwargs, id2label={0: "non-referral", 1: "referral"},
                      label2id={"non-referral": 0, "referral": 1})
    cfg._attn_implementation = "eager"
    model = VivitForVideoClassification(cfg).eval()
    sd = make_vivit_weights(cfg_kwargs, seed=wseed)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected, unexpected
    assert not missing, missing
    pix = make_synthetic_clips(batch, cfg_kwargs["num_frames"], cfg_kwargs["image_size"], seed=xseed)
    with torch.no_grad():
        out = model(pixel_values=torch.from_numpy(pix), output_hidden_states=not full)
    res = {"logits": out.logits.numpy()}
    if not full:
        res["hidden_states"] = np.stack([h.numpy() for h in out.hidden_states])
        res["pixel_values"] = pix
    res["weights_sha256"] = sha256_state(sd)
    res["pixel_sha256"] = hashlib.sha256(np.ascontiguousarray(pix).tobytes()).hexdigest()
    return res


VIVIT_TINY = dict(image_size=64, num_frames=4, tubelet_size=[2, 16, 16], num_channels=3, hidden_size=128,
                  num_hidden_layers=2, num_attention_heads=2, intermediate_size=256, hidden_act="gelu_fast",
                  layer_norm_eps=1e-6, qkv_bias=True)
VIVIT_B = dict(image_size=224, num_frames=32, tubelet_size=[2, 16, 16], num_channels=3, hidden_size=768,
               num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072, hidden_act="gelu_fast",
               layer_norm_eps=1e-6, qkv_bias=True)


def gen_vivit(skip_full):
    import numpy as np

    r = _vivit_golden(VIVIT_TINY, batch=3, wseed=0, xseed=1, full=False)
    np.savez_compressed(os.path.join(GOLDEN, "vivit_tiny.npz"), logits=r["logits"],
                        hidden_states=r["hidden_states"], pixel_values=r["pixel_values"],
                        config=json.dumps(VIVIT_TINY), weights_sha256=r["weights_sha256"])
    print("vivit_tiny logits", r["logits"])
    if skip_full:
        return
    r = _vivit_golden(VIVIT_B, batch=2, wseed=0, xseed=1, full=True)
    with open(os.path.join(GOLDEN, "vivit_full.json"), "w") as f:
        json.dump({"config": VIVIT_B, "batch": 2, "weights_seed": 0, "input_seed": 1,
                   "logits": r["logits"].tolist(), "weights_sha256": r["weights_sha256"],
                   "pixel_sha256": r["pixel_sha256"],
                   "oracle": "transformers VivitForVideoClassification (eager attention), fp32 CPU"}, f, indent=1)
    print("vivit_full logits", r["logits"])


def _timesformer_golden(cfg_kwargs, batch, wseed, xseed, full):
    import numpy as np
    import torch
    from transformers import TimesformerConfig, TimesformerForVideoClassification

    sys.path.insert(0, ROOT)
    from vclip_amd.weights import make_timesformer_weights, make_synthetic_clips, sha256_state

    cfg = TimesformerConfig(**cfg_kwargs, id2label={0: "non-referral", 1: "referral"},
                            label2id={"non-referral": 0, "referral": 1})
    model = TimesformerForVideoClassification(cfg).eval()
    sd = make_timesformer_weights(cfg_kwargs, seed=wseed)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected, unexpected
    assert not missing, missing
    pix = make_synthetic_clips(batch, cfg_kwargs["num_frames"], cfg_kwargs["image_size"], seed=xseed)
    with torch.no_grad():
        out = model(pixel_values=torch.from_numpy(pix), output_hidden_states=not full)
    res = {"logits": out.logits.numpy()}
    if not full:
        res["hidden_states"] = np.stack([h.numpy() for h in out.hidden_states])
        res["pixel_values"] = pix
    res["weights_sha256"] = sha256_state(sd)
    res["pixel_sha256"] = hashlib.sha256(np.ascontiguousarray(pix).tobytes()).hexdigest()
    return res


TSF_TINY = dict(image_size=64, patch_size=16, num_frames=4, num_channels=3, hidden_size=128, num_hidden_layers=2,
                num_attention_heads=2, intermediate_size=256, hidden_act="gelu", layer_norm_eps=1e-6, qkv_bias=True,
                attention_type="divided_space_time")
TSF_B = dict(image_size=224, patch_size=16, num_frames=8, num_channels=3, hidden_size=768, num_hidden_layers=12,
             num_attention_heads=12, intermediate_size=3072, hidden_act="gelu", layer_norm_eps=1e-6, qkv_bias=True,
             attention_type="divided_space_time")


def gen_timesformer(skip_full):
    import numpy as np

    r = _timesformer_golden(TSF_TINY, batch=3, wseed=0, xseed=1, full=False)
    np.savez_compressed(os.path.join(GOLDEN, "timesformer_tiny.npz"), logits=r["logits"],
                        hidden_states=r["hidden_states"], pixel_values=r["pixel_values"],
                        config=json.dumps(TSF_TINY), weights_sha256=r["weights_sha256"])
    print("timesformer_tiny logits", r["logits"])
    if skip_full:
        return
    r = _timesformer_golden(TSF_B, batch=2, wseed=0, xseed=1, full=True)
    with open(os.path.join(GOLDEN, "timesformer_full.json"), "w") as f:
        json.dump({"config": TSF_B, "batch": 2, "weights_seed": 0, "input_seed": 1,
                   "logits": r["logits"].tolist(), "weights_sha256": r["weights_sha256"],
                   "pixel_sha256": r["pixel_sha256"],
                   "oracle": "transformers TimesformerForVideoClassification, fp32 CPU"}, f, indent=1)
    print("timesformer_full logits", r["logits"])


def gen_baseline_batches():
    for name, fn, cfg, b in (("vivit_b8.json", _vivit_golden, VIVIT_B, 8),
                             ("timesformer_b16.json", _timesformer_golden, TSF_B, 16)):
        r = fn(cfg, batch=b, wseed=0, xseed=1, full=True)
        model = "VivitForVideoClassification (eager attention)" if fn is _vivit_golden else \
            "TimesformerForVideoClassification"
        with open(os.path.join(GOLDEN, name), "w") as f:
            json.dump({"config": cfg, "batch": b, "weights_seed": 0, "input_seed": 1,
                       "logits": r["logits"].tolist(), "weights_sha256": r["weights_sha256"],
                       "pixel_sha256": r["pixel_sha256"],
                       "baseline_config": "configs[1]" if fn is _vivit_golden else "configs[2]",
                       "oracle": f"transformers {model}, fp32 CPU"}, f, indent=1)
        print(name, r["logits"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only", choices=["sampling", "vivit", "timesformer", "baseline_batches"], default=None)
    a = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    if a.only in (None, "sampling"):
        gen_sampling()
    if a.only in (None, "vivit"):
        gen_vivit(a.skip_full)
    if a.only in (None, "timesformer"):
        gen_timesformer(a.skip_full)
    if a.only == "baseline_batches" or (a.only is None and not a.skip_full):
        gen_baseline_batches()  # BASELINE configs[1] / configs[2] at their own batch sizes


if __name__ == "__main__":
    main()
