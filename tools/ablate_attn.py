"""Timing-only ablations of the attention kernel: 1 no loop loads, 2 no exp, 4 no PV MFMA, 8 no QK MFMA."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import _lib
from tools.tune_gemm import timeit
lib = _lib.load()
f = lib.vc_attention_fwd_ablation
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_float,
              ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
B, S, H = 8, 3137, 12
qkv = torch.randn(25344, 2304, device="cuda").bfloat16()
o = torch.zeros(25344, 768, device="cuda", dtype=torch.bfloat16)
st = torch.cuda.current_stream().cuda_stream
fl = 4.0 * S * S * 64 * H * B
res = {}
abls = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,4,6,8,12,14,15,16,32,64,128,256,512,1024").split(",")]
for a in abls:
    f(qkv.data_ptr(), 2304, B, S, H, 0.125, o.data_ptr(), 768, a, st)
torch.cuda.synchronize()
for rnd in range(5):
    for a in abls:
        res.setdefault(a, []).append(timeit(lambda: f(qkv.data_ptr(), 2304, B, S, H, 0.125, o.data_ptr(), 768, a, st), 10))
print({a: f"{sorted(v)[2]*1e3:.0f}us {fl/sorted(v)[2]/1e9:.0f}TF" for a, v in res.items()})
# correct variants must agree with the shipped build (bits 1..15 are timing-only)
ref = None
for a in abls:
    if a & 15:
        continue
    o.zero_()
    f(qkv.data_ptr(), 2304, B, S, H, 0.125, o.data_ptr(), 768, a, st)
    torch.cuda.synchronize()
    if ref is None:
        ref = o.float().clone()
    print(f"abl {a}: max|diff| vs abl {abls[0]} = {(o.float() - ref).abs().max().item():.3e}")
