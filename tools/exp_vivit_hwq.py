"""ViViT-B B = 8 two-stream forward, eager and graph-replayed, re-created at several offsets of torch's stream
pool (k dummy torch.cuda.Stream() calls before the part streams are made): which runs land on shared
hardware queues (tools/hwq_probe.py) and serialize.
  python tools/exp_vivit_hwq.py [--trials 8]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from vclip_amd import streams  # noqa: E402
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--trials", type=int, default=8)
ap.add_argument("--tune", type=int, default=6, help="streams.TUNE_CANDIDATES")
ap.add_argument("--pats", default="0:0,-1:0", help="streams.TUNE_PRIORITIES for two parts (comma-separated p0:p1)")
ap.add_argument("--prios", default="default,0:0", help="comma-separated stream priority sets ('default' or p0:p1)")
a = ap.parse_args()
streams.TUNE_CANDIDATES[0] = a.tune
streams.TUNE_PRIORITIES[:] = [(lambda i, n, pr=tuple(int(v) for v in ps.split(":")): pr[i]) for ps in a.pats.split(",")]
dev = torch.device("cuda", 0)
pix = torch.from_numpy(make_synthetic_clips(8, 32, 224, seed=1)).to(dev)
m = create_model(num_frames=32, device=dev)
m.concurrent_streams = 2
ref = m.forward_logits(pix).clone()


def timeit():
    for _ in range(2):
        m.forward_logits(pix)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        m.forward_logits(pix)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 10 * 1e3


for k in range(a.trials):
    for _ in range(k):
        torch.cuda.Stream(device=dev)
    line = f"k={k}:"
    for ps in a.prios.split(","):
        m.stream_priorities = None if ps == "default" else [int(v) for v in ps.split(":")]
        m._streams = None
        streams._PICKED.clear()  # pick again (streams.pick_streams) after the offset
        m.__dict__.pop("_eager_sets", None)  # and tune the eager forward's sets again (streams.part_streams)
        m._graphs.clear()
        m.graph_replay = False
        te = timeit()
        m.graph_replay = True
        tg = timeit()
        same = torch.equal(m.forward_logits(pix), ref)
        line += f"  [{ps}] eager {8 / te * 1e3:.1f} graph {8 / tg * 1e3:.1f} clips/s{'' if same else ' LOGITS DIFFER'}"
    print(line, f" pick ok {dict(streams.PICK_STATUS)}", flush=True)
