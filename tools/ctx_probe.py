"""Why a GEMM runs slower inside the model than alone: time ViViT-B's fc2 (25344 x 768 x 3072, f32
residual epilogue) with HIP events around the fc2 launch only, under
  alone   -- fc2 repeated back to back (what tools/pp_check.py measures);
  after1  -- each fc2 right after the model's fc1 (writes fc2's 156-MB A operand);
  flush   -- each fc2 after a 512-MB memset (cold L2 / MALL, no dirty operand lines);
  idle    -- each fc2 after a 2 ms sleep kernel-free gap (clock recovers between launches).
The same for o_proj (25344 x 768 x 768) after the attention-output producer.  One JSON line per case.
  python tools/ctx_probe.py [--iters 20]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--M", type=int, default=25344)
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)
M = a.M


def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device="cuda", generator=g) * 2 - 1) * scale).bfloat16()


X = torch.randn(M, 768, device="cuda", generator=g)          # f32 residual stream
Y = rnd(M, 768)                                              # LayerNorm output
H = torch.zeros(M, 3072, device="cuda", dtype=torch.bfloat16)  # fc1 output = fc2's A
W1, b1 = rnd(3072, 768, scale=0.05), torch.randn(3072, device="cuda", generator=g) * 0.1
W2, b2 = rnd(768, 3072, scale=0.05), torch.randn(768, device="cuda", generator=g) * 0.1
Wo, bo = rnd(768, 768, scale=0.05), torch.randn(768, device="cuda", generator=g) * 0.1
flushbuf = torch.empty(512 * 1024 * 1024 // 4, device="cuda", dtype=torch.float32)


def fc1():
    ops.gemm(Y, W1, b1, "bias_gelu_tanh", H)


def fc2():
    ops.gemm(H, W2, b2, "bias_resid_f32", X)


def oproj():
    ops.gemm(Y, Wo, bo, "bias_resid_f32", X)


def flush():
    flushbuf.fill_(1.0)


def idle():
    torch.cuda.synchronize()
    time.sleep(0.002)


def run(name, op, pre):
    ts = []
    for i in range(a.iters + 3):
        if pre is not None:
            pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        op()
        e1.record()
        e1.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    print(json.dumps({"case": name, "us_med": round(ts[len(ts) // 2], 1), "us_min": round(ts[0], 1),
                      "us_max": round(ts[-1], 1)}), flush=True)


fc1()
torch.cuda.synchronize()
for name, op, pre in (("fc2_alone", fc2, None), ("fc2_after_fc1", fc2, fc1), ("fc2_after_flush", fc2, flush),
                      ("fc2_after_idle", fc2, idle), ("oproj_alone", oproj, None), ("oproj_after_fc1", oproj, fc1),
                      ("oproj_after_flush", oproj, flush), ("oproj_after_idle", oproj, idle),
                      ("fc1_alone", fc1, None), ("fc1_after_flush", fc1, flush)):
    run(name, op, pre)
