"""Does a kernel on stream b get dispatched while a big kernel on stream a is still being dispatched?
A = vc_spin with 4x the GPU's one-wave slots (about four rounds of short sleeps) on stream a, then
B = one one-wave workgroup on stream b; tB / tA = B's completion over A's (host clock).  Small: b's
workgroups are dispatched beside a's (different pipes / an arbiter that interleaves); near 1: b waits
for a's whole dispatch.  Pairs of torch pool streams at several pool offsets and priorities.
  python tools/hwq_pipe_probe.py"""
import sys
import time

import torch

sys.path.insert(0, ".")
from vclip_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
NB = 4 * 256 * 32
ITERS = 24


def probe(a, b):
    res = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(a):
            ops.spin(ITERS, dev, NB)
        with torch.cuda.stream(b):
            ops.spin(1, dev, 1)
        b.synchronize()
        tb = time.perf_counter() - t0
        a.synchronize()
        ta = time.perf_counter() - t0
        res.append((tb / ta, ta))
    return min(r[0] for r in res), min(r[1] for r in res)


with torch.cuda.stream(torch.cuda.Stream(device=dev)):
    ops.spin(ITERS, dev, NB)
torch.cuda.synchronize()
for pa, pb in ((0, 0), (-1, 0), (0, -1)):
    line = f"priorities a={pa:2d} b={pb:2d}:"
    for k in range(8):
        a = torch.cuda.Stream(device=dev, priority=pa)
        b = torch.cuda.Stream(device=dev, priority=pb)
        r, ta = probe(a, b)
        r2, _ = probe(b, a)
        line += f"  {r:.2f}/{r2:.2f}"
    print(line, f"  (A {ta * 1e3:.2f} ms; ratio a->b / b->a)", flush=True)
