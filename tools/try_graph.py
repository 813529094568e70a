"""A/B: ViViT-B B=8 forward launched eagerly vs replayed from a captured HIP graph
(torch.cuda.CUDAGraph over the same ctypes launches), interleaved rounds in one process;
checks the replayed logits are bit-identical.

  python tools/try_graph.py [--rounds 5] [--iters 10] [--batch 8]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    dev = "cuda"
    model = create_model(num_frames=32, device=dev)
    pix = torch.from_numpy(make_synthetic_clips(a.batch, 32, 224, seed=1)).to(dev)
    eager = lambda: model.forward_logits(pix)  # noqa: E731
    ref = eager().clone()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        eager()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            out = model.forward_logits(pix)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    print("graph logits bit-identical:", torch.equal(out, ref), flush=True)
    cands = {"eager": eager, "graph": g.replay}
    times = {k: [] for k in cands}
    for _ in range(a.rounds):
        for k, f in cands.items():
            times[k].append(timeit(f, a.iters))
    for k, ts in times.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"{k:6s} {med:7.3f} ms/step  {a.batch / med * 1e3:7.1f} clips/s (min {ts[0]:.3f})", flush=True)


if __name__ == "__main__":
    main()
