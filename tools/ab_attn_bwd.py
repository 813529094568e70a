"""Interleaved timing of the attention backward (vc_attention_bwd: prep + dK/dV + dQ) of several
libvclip.so builds in ONE process (cdna_hip_programming.md rule 24), on ViViT-B train-step inputs
(default B=4, S=3137, H=12): the forward with log-sum-exp from the first library, then each
library's backward; outputs compared bit for bit with the first library's.
  python tools/ab_attn_bwd.py libA.so libB.so ... [--B 4] [--rounds 10] [--iters 5]"""
import argparse
import ctypes
import os

import numpy as np
import torch

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--B", type=int, default=4)
ap.add_argument("--S", type=int, default=3137)
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
B, S, H = a.B, a.S, 12
g = torch.Generator(device="cuda").manual_seed(0)
qkv = (torch.randn(B * S, 3 * H * 64, device="cuda", generator=g) * 1.5).bfloat16()
dout = (torch.randn(B * S, H * 64, device="cuda", generator=g)).bfloat16()
st = torch.cuda.current_stream()
P, I64, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
libs = [ctypes.CDLL(os.path.abspath(p), mode=os.RTLD_LOCAL) for p in a.libs]
fwd = libs[0].vc_attention_fwd_lse
fwd.restype = ctypes.c_int
fwd.argtypes = [P, I64, I64, I64, I64, I64, F, ctypes.c_int, P, I64, P, P]
out = torch.zeros(B * S, H * 64, device="cuda", dtype=torch.bfloat16)
lse = torch.zeros(B * H * S, device="cuda", dtype=torch.float32)
assert fwd(qkv.data_ptr(), 3 * H * 64, B, S, H, 64, 0.125, 0, out.data_ptr(), H * 64, lse.data_ptr(),
           st.cuda_stream) == 0
fns = []
for lib in libs:
    f = lib.vc_attention_bwd
    f.restype = ctypes.c_int
    f.argtypes = [P, I64, P, I64, P, I64, P, P, I64, I64, I64, I64, P, I64, P]
    fns.append(f)
delta = torch.zeros(B * H * S, device="cuda", dtype=torch.float32)
grads = []
for f in fns:
    d = torch.zeros(B * S, 3 * H * 64, device="cuda", dtype=torch.bfloat16)
    assert f(qkv.data_ptr(), 3 * H * 64, out.data_ptr(), H * 64, dout.data_ptr(), H * 64, lse.data_ptr(),
             delta.data_ptr(), B, S, H, 64, d.data_ptr(), 3 * H * 64, st.cuda_stream) == 0
    grads.append(d)
torch.cuda.synchronize()
for p, d in zip(a.libs, grads):
    print(f"{p:48s} bit-identical to first: {torch.equal(d, grads[0])}", flush=True)
times = [[] for _ in fns]
d = grads[0]
for r in range(a.rounds):
    for i in (range(len(fns)) if r % 2 == 0 else reversed(range(len(fns)))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fns[i](qkv.data_ptr(), 3 * H * 64, out.data_ptr(), H * 64, dout.data_ptr(), H * 64, lse.data_ptr(),
                   delta.data_ptr(), B, S, H, 64, d.data_ptr(), 3 * H * 64, st.cuda_stream)
        e1.record()
        e1.synchronize()
        times[i].append(e0.elapsed_time(e1) * 1000 / a.iters)
flop = 2 * 4.0 * B * H * S * S * 64  # algorithmic: dV, dP, dK, dQ
for p, t in zip(a.libs, times):
    t = np.array(t)
    print(f"{p:48s} median {np.median(t):8.2f} us  min {t.min():8.2f}  ({flop / np.median(t) / 1e6:.0f} TF/s algorithmic)",
          flush=True)
