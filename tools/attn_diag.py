"""DIAGNOSTIC: time the ping-pong attention kernel with parts removed (timing only)."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import _lib
lib = _lib.load()
f = lib.vc_attention_fwd_diag
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
              ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
B, S, H = 8, 3137, 12
qkv = (torch.randn(25344, 2304, device="cuda") * 0.5).bfloat16()
o = torch.zeros(25344, 768, device="cuda", dtype=torch.bfloat16)
st = torch.zeros(64 * 8 * 64 * 4 + 64 * 8, dtype=torch.int64, device="cuda")
names = {0: "full", 2: "no fragment reads", 4: "no exp2", 8: "no MFMA", 6: "no reads+exp", 12: "no exp+MFMA",
         14: "no reads+exp+MFMA"}
for rnd in range(2):
    for d, nm in names.items():
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            f(qkv.data_ptr(), 2304, B, S, H, o.data_ptr(), 768, st.data_ptr(), d, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            assert f(qkv.data_ptr(), 2304, B, S, H, o.data_ptr(), 768, st.data_ptr(), d, s) == 0
        e1.record()
        torch.cuda.synchronize()
        print(f"{nm:24s} {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us", flush=True)
