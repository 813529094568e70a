"""DIAGNOSTIC: per-phase s_memtime stamps of the ping-pong attention kernel (first 64 WGs).
Stamp k of phase p: 0 after the DMA issue, 1 after the fragment prefetch (V) / MFMA issue (M),
2 before the phase's vmcnt wait, 3 after the barrier."""
import ctypes, os, sys
import numpy as np
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
for _ in range(4):
    assert f(qkv.data_ptr(), 2304, B, S, H, o.data_ptr(), 768, st.data_ptr(), 1, torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
a = st.cpu().numpy()
lead = a[64 * 8 * 64 * 4:].reshape(64, 8)
a = a[:64 * 8 * 64 * 4].reshape(64, 8, 64, 4)  # [wg][wave][phi+1][k]
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/attn_stamps.npy", a)
# phases 10..40 (phi = index - 1); start of phase phi = stamp 3 of phase phi-1
for kind in ("M", "V"):
    rows = []
    for wg in range(64):
        for w in range(8):
            for idx in range(11, 41):
                phi = idx - 1
                is_m = (phi % 2 == 1) == bool(lead[wg, w])
                if (kind == "M") != is_m:
                    continue
                s0 = a[wg, w, idx - 1, 3]
                st4 = a[wg, w, idx]
                rows.append([st4[0] - s0, st4[1] - st4[0], st4[2] - st4[1], st4[3] - st4[2], st4[3] - s0])
    r = np.median(np.array(rows), axis=0)
    print(f"{kind} phase median ticks: stage {r[0]:.0f}  {'mfma-issue' if kind == 'M' else 'prefetch'} {r[1]:.0f}  "
          f"{'mask' if kind == 'M' else 'softmax'} {r[2]:.0f}  wait+barrier {r[3]:.0f}  total {r[4]:.0f}")
