"""A/B of the f32-residual prefetch in the 128x128 GEMM (cfg 5 = prefetch, cfg 8 = without):
isolated o_proj / fc2 at ViViT-B B=8 and the whole forward with every residual GEMM forced to
one or the other (interleaved rounds, one process); outputs must be bit-identical."""
import sys
import time

import torch

sys.path.insert(0, ".")
from vclip_amd import ops  # noqa: E402
from vclip_amd.vivit import create_model  # noqa: E402
from vclip_amd.weights import make_synthetic_clips  # noqa: E402
from tools.tune_gemm import timeit  # noqa: E402

dev = torch.device("cuda", 0)
CFGS = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "5,8").split(",")]
g = torch.Generator(device=dev).manual_seed(0)
M = 25344
for name, N, K in [("o_proj", 768, 768), ("fc2", 768, 3072)]:
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device=dev, generator=g) * 0.1
    X0 = torch.randn(M, N, device=dev, generator=g)
    outs = {}
    for c in CFGS:
        X = X0.clone()
        ops.gemm(A, W, b, "bias_resid_f32", X, cfg=c)
        outs[c] = X
    print(name, "bit-identical:", all(torch.equal(outs[CFGS[0]], o) for o in outs.values()), flush=True)
    X = X0.clone()
    res = {c: [] for c in CFGS}
    for _ in range(5):
        for c in CFGS:
            res[c].append(timeit(lambda: ops.gemm(A, W, b, "bias_resid_f32", X, cfg=c), 20))
    print(name, {c: f"{sorted(v)[2] * 1e3:.1f}us" for c, v in res.items()}, flush=True)

orig = ops.gemm
mode = {"cfg": -1}


def patched(a, w, bias, epilogue, out, *args, **kw):
    if epilogue == "bias_resid_f32" and kw.get("cfg", -1) == -1:
        kw["cfg"] = mode["cfg"]
    return orig(a, w, bias, epilogue, out, *args, **kw)


ops.gemm = patched
pix = torch.from_numpy(make_synthetic_clips(8, 32, 224, seed=1)).to(dev)
m = create_model(num_frames=32, device=dev)
lg = {}
for c in CFGS:
    mode["cfg"] = c
    lg[c] = m.forward_logits(pix).clone()
print("model logits bit-identical:", all(torch.equal(lg[CFGS[0]], o) for o in lg.values()), flush=True)
res = {c: [] for c in CFGS}
for _ in range(6):
    for c in CFGS:
        mode["cfg"] = c
        for _ in range(2):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.forward_logits(pix)
        torch.cuda.synchronize()
        res[c].append((time.perf_counter() - t0) / 10 * 1e3)
for c, ts in res.items():
    ts.sort()
    print(f"model resid cfg {c}: median {ts[3]:.3f} ms/step ({8 / ts[3] * 1e3:.1f} clips/s)", flush=True)
