"""A/B of the attention forward with and without the sched_group_barrier MFMA/VALU interleave
(ablation bit 32, a correct variant), interleaved rounds in one process, at B = 8 and B = 4."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import _lib
from tools.tune_gemm import timeit
lib = _lib.load()
f = lib.vc_attention_fwd_ablation
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_float,
              ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
S, H = 3137, 12
st = torch.cuda.current_stream().cuda_stream
for B in (8, 4):
    rows = (B * S + 128 + 255) // 256 * 256
    qkv = torch.randn(rows, 2304, device="cuda").bfloat16()
    o = torch.zeros(rows, 768, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * S * S * 64 * H * B
    res = {}
    for a in (0, 32):
        f(qkv.data_ptr(), 2304, B, S, H, 0.125, o.data_ptr(), 768, a, st)
    torch.cuda.synchronize()
    for rnd in range(11):
        for a in (0, 32):
            res.setdefault(a, []).append(timeit(lambda: f(qkv.data_ptr(), 2304, B, S, H, 0.125, o.data_ptr(), 768, a, st), 20))
    print(B, {a: f"{sorted(v)[5]*1e3:.1f}us {fl/sorted(v)[5]/1e9:.0f}TF (min {sorted(v)[0]*1e3:.1f})" for a, v in res.items()})
