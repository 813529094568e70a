"""Forward replayed from a captured HIP graph vs eager enqueue, interleaved rounds in one process.

usage: python tools/exp_graph.py [vivit|timesformer|swin] [B] [graph3,graph4,graph2_rs]
Each variant: the model's own forward_logits (1 or 2 concurrent HIP streams) enqueued eagerly, or
the same call captured once into a torch.cuda.CUDAGraph (hipGraph) and replayed.  Logits must be
bit-identical; every round's clips/s is printed (the box spread matters)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

fam = sys.argv[1] if len(sys.argv) > 1 else "vivit"
dev = torch.device("cuda", 0)
if fam == "vivit":
    from vclip_amd.vivit import create_model
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    m = create_model(num_frames=32, device=dev)
    pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
elif fam == "timesformer":
    from vclip_amd.timesformer import create_model
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    m = create_model(num_frames=8, device=dev)
    pix = torch.from_numpy(make_synthetic_clips(B, 8, 224, seed=1)).to(dev)
elif fam == "swin":
    from vclip_amd.swin3d import create_model
    from vclip_amd.weights import make_synthetic_video
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    m = create_model(model_size="tiny", device=dev)
    pix = torch.from_numpy(make_synthetic_video(B, 32, 224, seed=1)).to(dev)
else:
    raise SystemExit(f"unknown family {fam}")
m.eval()


def eager(ns):
    def f():
        m.concurrent_streams = ns
        return m.forward_logits(pix)
    return f


def graphed(ns):
    m.concurrent_streams = ns
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            m.forward_logits(pix)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = m.forward_logits(pix)
    # the graph addresses the model's workspaces: hold them, since a later capture's warm-up may
    # drop the model's workspace cache (TimeSformer B=16 over 1-4 streams makes 10 part workspaces,
    # past the cache's 8) and torch.cuda.graph empties the allocator cache at capture start, which
    # would unmap them under this graph (an illegal-address fault in round 3's first version)
    keep = (m._packed, m._ws, getattr(m, "_split_out", None), getattr(m, "_bias_cache", None))

    def f(keep=keep):
        g.replay()
        return out
    return f


def graphed_with(ns, **attrs):
    """a graph captured with model attributes set (e.g. ViViT round_split), restored after capture"""
    old = {k: getattr(m, k) for k in attrs}
    for k, v in attrs.items():
        setattr(m, k, v)
    f = graphed(ns)
    for k, v in old.items():
        setattr(m, k, v)
    return f


ref = eager(1)().clone()
extra = sys.argv[3].split(",") if len(sys.argv) > 3 else []
VAR = {"eager2": eager(2), "graph2": graphed(2)} if extra else \
    {"eager1": eager(1), "eager2": eager(2), "graph1": graphed(1), "graph2": graphed(2)}
for v in extra:  # graph3, graph4, graph2_rs (ViViT round_split)
    if v.startswith("graph") and v[5:].isdigit():
        VAR[v] = graphed(int(v[5:]))
    elif v == "graph2_rs":
        VAR[v] = graphed_with(2, round_split=True)
for k, f in VAR.items():
    got = f().clone()
    torch.cuda.synchronize()
    print(k, "bit-identical" if torch.equal(got, ref) else f"DIFF {float((got - ref).abs().max()):.3e}", flush=True)
res = {v: [] for v in VAR}
for rnd in range(6):
    for k, f in VAR.items():
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(12):
            f()
        torch.cuda.synchronize()
        res[k].append(B * 12 / (time.perf_counter() - t0))
    print("round", rnd, {k: round(v[-1], 1) for k, v in res.items()}, flush=True)
for v, x in res.items():
    print(f"{fam} B={B} {v}: median {np.median(x):.1f} min {min(x):.1f} max {max(x):.1f}", flush=True)
