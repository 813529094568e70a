"""Where a ping-pong GEMM launch spends its time: cfg 18 = the cfg 8 kernel (gemm_pp_kernel) with
s_memrealtime stamps (100 MHz, chip-wide) per workgroup and wave group at entry, after the prologue
wait, after the main loop, after the epilogue stores issued and after they drained, plus the shader
cycles between entry and drain (s_memtime) -> per-segment percentiles for the first and the later
rounds of workgroups, the launch ramp and the kernel span.

  python tools/gemm_stamps.py [--shapes 12800x2304x768,12800x768x3072] [--iters 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="12800x2304x768:bias,12800x3072x768:bias_gelu_tanh,12800x768x3072:bias_resid_f32,"
                                     "12800x768x768:bias_resid_f32")
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--ppd", default="12800x2304x768:bias,25344x2304x768:bias,12800x3072x768:bias_gelu_tanh",
                help="shapes for the persistent deferred-store kernel (cfg 15): per-tile times")
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)


def pct(x):
    x = np.asarray(x, dtype=np.float64)
    return {"p10": round(float(np.percentile(x, 10)), 2), "p50": round(float(np.percentile(x, 50)), 2),
            "p90": round(float(np.percentile(x, 90)), 2)}


for shp in a.shapes.split(","):
    dims, epi = shp.split(":")
    M, N, K = (int(v) for v in dims.split("x"))
    A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    f32 = epi == "bias_resid_f32"
    init = torch.randn(M, N, device="cuda", generator=g) if f32 else torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    out = init.clone()
    ref = init.clone()
    ops.gemm(A, W, b, epi, ref, cfg=8)
    nwg = (M // 256) * (N // 256)
    st = torch.zeros(nwg * 2 * 8, dtype=torch.int64, device="cuda")
    for it in range(a.iters):
        if f32:
            out.copy_(init)
        ops.gemm(A, W, b, epi, out, aux=st, cfg=18)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), "cfg 18 must compute what cfg 8 computes"
    s = st.view(nwg, 2, 8).cpu().numpy().astype(np.int64)
    t0 = s[:, :, 0].min()
    start = (s[:, 0, 0] - t0) / 100.0  # us
    span = (s[:, :, 4].max() - t0) / 100.0
    # rounds: workgroups that started after the first finished
    first_end = (s[:, :, 4].min() - t0) / 100.0
    r1 = start < first_end
    seg = lambda i, j: (s[:, :, j] - s[:, :, i]) / 100.0  # noqa: E731
    clock = s[:, :, 5] / ((s[:, :, 4] - s[:, :, 0]) * 10.0)  # cycles per ns = GHz
    out_line = {"shape": [M, N, K], "epilogue": epi, "tiles": nwg, "span_us": round(float(span), 2),
                "wall_from_events_note": "span = last drain - first entry (one launch)",
                "first_round": int(r1.sum()), "later_count": int((~r1).sum()),
                "start_us_later_rounds": pct(start[~r1]) if (~r1).any() else None}
    for name, mask in (("round1", r1), ("later", ~r1)):
        if not mask.any():
            continue
        out_line[name] = {"prologue_us": pct(seg(0, 1)[mask].ravel()), "main_us": pct(seg(1, 2)[mask].ravel()),
                          "epi_issue_us": pct(seg(2, 3)[mask].ravel()), "drain_us": pct(seg(3, 4)[mask].ravel()),
                          "total_us": pct(seg(0, 4)[mask].ravel()), "clock_ghz": pct(clock[mask].ravel())}
    print(json.dumps(out_line), flush=True)
    del A, W, b, out, ref, st, init
    torch.cuda.empty_cache()


# cfg 19 = cfg 15 (persistent, deferred stores) with s_memrealtime per workgroup at entry, after each tile's main loop, end
for shp in (a.ppd.split(",") if a.ppd else []):
    dims, epi = shp.split(":")
    M, N, K = (int(v) for v in dims.split("x"))
    A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    out = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    ref = out.clone()
    ops.gemm(A, W, b, epi, ref, cfg=8)
    st = torch.zeros(256 * 16, dtype=torch.int64, device="cuda")
    for _ in range(a.iters):
        st.zero_()
        ops.gemm(A, W, b, epi, out, aux=st, cfg=19)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), "cfg 15 must compute what cfg 8 computes"
    s = st.view(256, 16).cpu().numpy().astype(np.int64)
    s = s[s[:, 0] > 0]
    t0 = s[:, 0].min()
    first = (s[:, 1] - s[:, 0]) / 100.0
    tiles = []
    for wg in s:
        ts = [t for t in wg[1:15] if t > 0]
        tiles += [(ts[i + 1] - ts[i]) / 100.0 for i in range(len(ts) - 1)]
    tail = (s[:, 15] - np.array([max(t for t in wg[1:15] if t > 0) for wg in s])) / 100.0
    print(json.dumps({"ppd_shape": [M, N, K], "epilogue": epi, "workgroups": int(len(s)),
                      "span_us": round(float((s[:, 15].max() - t0) / 100.0), 2),
                      "start_spread_us": pct((s[:, 0] - t0) / 100.0), "first_tile_us": pct(first),
                      "next_tiles_us": pct(tiles) if tiles else None, "last_epilogue_us": pct(tail)}), flush=True)
    del A, W, b, out, ref, st
    torch.cuda.empty_cache()
