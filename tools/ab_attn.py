"""A/B the attention kernel of several libvclip builds, interleaved in one process.

  python tools/ab_attn.py [lib.so ...]     (default: the in-tree library + every ab/*/libvclip.so)
  ABL=32,16 python tools/ab_attn.py        (also the in-tree library's ablation variants)
"""
import ctypes
import glob
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vclip_amd import _lib  # noqa: E402
from tools.tune_gemm import timeit  # noqa: E402

_lib.load()  # torch + the in-tree library first (one HIP runtime)
paths = sys.argv[1:] or [os.path.join(ROOT, "ai-laryngeal-video-based-classifier_amd", "libvclip.so")] + sorted(
    glob.glob(os.path.join(ROOT, "ab", "*", "libvclip.so")))
B, S, H = 8, 3137, 12
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(25344, 2304, device="cuda", generator=g).bfloat16()
st = torch.cuda.current_stream().cuda_stream
fl = 4.0 * S * S * 64 * H * B
fns, outs = {}, {}
for p in paths:
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    f = lib.vc_attention_fwd
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                  ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    o = torch.zeros(25344, 768, device="cuda", dtype=torch.bfloat16)
    name = os.path.basename(os.path.dirname(p))
    fns[name] = (lambda f=f, o=o: f(qkv.data_ptr(), 2304, B, S, H, 64, 0.125, 0, o.data_ptr(), 768, st))
    outs[name] = o
tree = _lib.load()
fa = tree.vc_attention_fwd_ablation
fa.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_float,
               ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
for a in [int(x) for x in os.environ.get("ABL", "").split(",") if x]:
    o = torch.zeros(25344, 768, device="cuda", dtype=torch.bfloat16)
    fns[f"tree_abl{a}"] = (lambda a=a, o=o: fa(qkv.data_ptr(), 2304, B, S, H, 0.125, o.data_ptr(), 768, a, st))
    outs[f"tree_abl{a}"] = o
for f in fns.values():
    assert f() == 0
torch.cuda.synchronize()
base = next(iter(outs.values()))
for k, o in outs.items():
    print(f"{k}: max|diff| vs first {(o.float() - base.float()).abs().max().item():.4f}")
res = {k: [] for k in fns}
for rnd in range(int(os.environ.get("ROUNDS", "7"))):
    for k, f in fns.items():
        res[k].append(timeit(f, 10))
for k, v in res.items():
    v.sort()
    print(f"{k:40s} median {v[len(v) // 2] * 1e3:7.1f} us  {fl / v[len(v) // 2] / 1e9:6.0f} TF   min {v[0] * 1e3:7.1f} us")
