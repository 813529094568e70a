"""Forward throughput with the batch split over S concurrent HIP streams (independent clips),
each with its own model workspace, vs one stream; ViViT-B 32x224^2."""
import sys
import time

import torch

sys.path.insert(0, ".")
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
pix = torch.from_numpy(make_synthetic_clips(B, 32, 224, seed=1)).to(dev)
models = [create_model(num_frames=32, device=dev) for _ in range(4)]
streams = [torch.cuda.Stream(device=dev) for _ in range(4)]


def run(ns):
    cur = torch.cuda.current_stream()
    parts = torch.chunk(pix, ns)
    for i in range(ns):
        streams[i].wait_stream(cur)
        with torch.cuda.stream(streams[i]):
            models[i].forward_logits(parts[i])
    for i in range(ns):
        cur.wait_stream(streams[i])


ref = models[0].forward_logits(pix).clone()
for ns in (1, 2, 4):
    out = torch.cat([models[i].forward_logits(p) for i, p in enumerate(torch.chunk(pix, ns))])
    assert (out - ref).abs().max() < 1e-5
res = {}
for rnd in range(3):
    for ns in (1, 2, 4):
        for _ in range(3):
            run(ns)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            run(ns)
        torch.cuda.synchronize()
        res.setdefault(ns, []).append(B * 20 / (time.perf_counter() - t0))
print({ns: f"{sorted(v)[1]:.1f} clips/s" for ns, v in res.items()})
