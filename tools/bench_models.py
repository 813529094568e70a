"""Forward throughput of the non-headline model families at their BASELINE configs
(SURVEY.md §8(d)): TimeSformer-B 8f B=16 (cfg3), Video Swin-T 32f (cfg4: B=4 per GPU),
plus ViViT-B for reference.

  python tools/bench_models.py [--model timesformer] [--batch 16] [--steps 20] [--warmup 3]

Prints one JSON line per model: clips/s, ms/step, model TFLOP/s (GFLOP/clip from §8(d)).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GFLOP = {"vivit": 903.05, "timesformer": 391.66, "swin3d_t": 175.53, "resnet3d_50": 349.03}


def build(name, batch, dev):
    from vclip_amd.weights import make_synthetic_clips
    if name == "swin3d_t":
        from vclip_amd.swin3d import create_model
        from vclip_amd.weights import make_synthetic_video
        m = create_model(model_size="tiny", device=dev)
        return m, torch.from_numpy(make_synthetic_video(batch, 32, 224, seed=1)).to(dev)
    if name == "resnet3d_50":
        from vclip_amd.resnet3d import create_model
        from vclip_amd.weights import make_synthetic_video
        m = create_model(device=dev)
        return m, torch.from_numpy(make_synthetic_video(batch, 32, 224, seed=1)).to(dev)
    if name == "vivit":
        from vclip_amd.vivit import create_model
        m = create_model(num_frames=32, device=dev)
        T = 32
    else:
        from vclip_amd.timesformer import create_model
        m = create_model(num_frames=8, device=dev)
        T = 8
    pix = torch.from_numpy(make_synthetic_clips(batch, T, 224, seed=1)).to(dev)
    return m, pix


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="timesformer")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name in a.model.split(","):
        m, pix = build(name, a.batch, dev)
        for _ in range(a.warmup):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        cps = a.batch * a.steps / dt
        print(json.dumps({"model": name, "batch": a.batch, "clips_per_s": round(cps, 2),
                          "ms_per_step": round(dt / a.steps * 1e3, 3),
                          "model_tflops": round(GFLOP[name] * cps / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
