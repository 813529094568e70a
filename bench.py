"""Headline benchmark: clips/sec of the ViViT-B/16x2 forward, 32x224^2 clips, batch 8
per GPU, bf16 MFMA compute (BASELINE.json `metric`, configs[1]), plus the logit
max-abs-error vs the fp32 CPU reference and a roofline line for the dominant kernel.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]
  python bench.py --mode train [...]   # BASELINE configs[4]: ViViT-B train step (fwd + bwd +
                                       # AdamW) bf16, 4 clips per GPU, RCCL gradient all-reduce
  python bench.py --mode timesformer   # BASELINE configs[2]: TimeSformer-B 8f, 16 clips per GPU
  python bench.py --mode swin          # BASELINE configs[3]: Video Swin-T 32f, 4 clips per GPU
  python bench.py --mode resnet3d      # the resnet50-3d-video family: ResNet3D-50 32f, 4 clips per GPU

One process per GPU (torch.distributed.run for N > 1, backend nccl = RCCL).  Clips
shard as independent data-parallel units: each rank runs its own batch and no
collective touches the hot path; a barrier + device sync bracket the
timed region and the MAX elapsed over ranks is used.  Inputs (synthetic, seeded, per
rank) are resident in HBM before timing starts.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vclip_amd import streams as vstreams  # noqa: E402

ATTN_GFLOP_PER_CLIP_LAYER = 4.0 * 3137 * 3137 * 64 * 12 / 1e9  # QK^T + PV, 30.23 GF
VIVIT_GFLOP_PER_CLIP = 903.05   # measured with torch.utils.flop_counter on the HF model
ATTN_GFLOP_PER_CLIP = 362.77
ATTN_IO_BYTES_PER_CLIP = 3137 * 768 * 2 * 4  # q,k,v read + o written once, bf16
# attention backward, compulsory per clip and layer: q,k,v, o and dO read, dq,dk,dv written (bf16), the
# log-sum-exp read and delta = rowsum(dO * o) written and read (f32 per query and head)
TRAIN_ATTN_IO_BYTES_PER_CLIP = 3137 * 768 * 2 * (3 + 1 + 1 + 3) + 3137 * 12 * 4 * 3
PEAK_BF16_TFLOPS = 2500.0       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
# the headline's dominant kernel as rocprofv3 names it (template args: no rebase test build, no
# lse, bf16 operands) -- the key of its counters in profiles/rNN_*_{traffic,pmc}.json
ATTN_KERNEL = "attn_fwd_d64_kernel<false, false, 0>"


def _build_id():
    from vclip_amd.build import source_hash
    return source_hash()


def _same_build(pattern: str, mode: str):
    """The committed profiles/<pattern> summary of THIS tree's build ("build" =
    vclip_amd.build.source_hash of the sources it was measured on) AND of this bench mode ("mode":
    the workload the profiled command ran, stamped by tools/collect_profiles.py), newest by the
    numbers in its name; (None, reason) when there is none, or when two such files tie: a roofline
    line never cites counters of another build or of another workload."""
    import glob
    import re
    me = _build_id()
    fs = []
    dirs = [os.path.join(ROOT, "profiles")] + [d for d in os.environ.get("VCLIP_PROFILES", "").split(":") if d]
    seen = set()
    for f in sorted(f for d in dirs for f in glob.glob(os.path.join(d, pattern))):
        if os.path.basename(f) in seen:
            continue
        seen.add(os.path.basename(f))
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("build") == me and d.get("mode") == mode:
            fs.append((f, d))
    if not fs:
        return None, f"no {pattern} profile of this build and mode {mode!r} under profiles/"
    key = lambda fd: [int(x) for x in re.findall(r"\d+", os.path.basename(fd[0]))]  # noqa: E731
    best = max(key(fd) for fd in fs)
    top = [fd for fd in fs if key(fd) == best]
    if len(top) > 1:
        return None, "ambiguous: " + ", ".join(sorted(_cite(f) for f, _ in top))
    return top[0]


def _cite(f: str) -> str:
    """how a line cites a summary: profiles/<name> (a session's own summaries are collected into
    profiles/ under the same name: tools/profile_round.sh, tools/collect_profiles.py)"""
    return "profiles/" + os.path.basename(f)


def measured_traffic(kernels, mode: str = "fwd"):
    """HBM bytes per launch of `kernels` (one rocprofv3 kernel name, or a list whose per-launch bytes
    add up) from the FETCH_SIZE x2 + WRITE_SIZE passes over this bench mode's command
    (tools/profile_round.sh -> profiles/rNN_*_traffic.json) of this build: (bytes, source) or
    (None, reason)."""
    f, d = _same_build("r*_traffic.json", mode)
    if not f:
        return None, d
    ks = [kernels] if isinstance(kernels, str) else list(kernels)
    if any(k not in d["kernels"] for k in ks):
        return None, f"{_cite(f)} has no entry for {ks}"
    return sum(d["kernels"][k]["hbm_bytes_per_launch"] for k in ks), _cite(f)


def measured_pmc(kernel: str, mode: str = "fwd"):
    """Per-launch PMC averages of `kernel` for this build and mode (profiles/rNN_*_pmc.json), else
    (None, reason)."""
    f, d = _same_build("r*_pmc.json", mode)
    if not f:
        return None, d
    if kernel not in d.get("kernels", {}):
        return None, f"{_cite(f)} has no entry for {kernel}"
    return d["kernels"][kernel], _cite(f)


def pmc_rates(pmc):
    """(MFMA busy, VALU instructions per MFMA) from a kernel's PMC averages:
    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); SQ_INSTS_VALU counts the MFMAs."""
    if not pmc:
        return None, None
    return (round(pmc["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * pmc["GRBM_GUI_ACTIVE"] / 8), 4),
            round(pmc["SQ_INSTS_VALU"] / pmc["SQ_INSTS_MFMA"], 3))


def _spawn_world(n: int) -> int:
    """`bench.py --gpus N` without a launcher: re-run this command under torch.distributed.run
    with N local ranks (one process per GPU, rendezvous on 127.0.0.1).  The parent touches no
    GPU (the children initialise HIP); it waits and returns the launcher's exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(lr)
        dist.init_process_group("nccl", device_id=torch.device("cuda", lr))
        return dist, dist.get_rank(), ws, lr
    return None, 0, 1, 0


def _graph_used(model, a) -> bool:
    """the headline replayed a captured hipGraph (--graph 1 on a model with graph replay)"""
    return bool(a.graph) and getattr(model, "_graphs", None) is not None


def _stream_tuning(model):
    """(priorities, ms per replay) of each stream set the headline's part graphs were timed on at capture
    (streams.GraphReplay._tune; the fastest is the one replayed), or None (no split graph)"""
    g = getattr(model, "_graphs", None)
    return None if g is None or g.tune_log is None else [{"priorities": list(p), "ms": t} for p, t in g.tune_log]


def timed_loop(step, steps: int, warmup: int, dist=None, sync=None):
    """W untimed warm-up steps, then exactly `steps` timed steps bracketed by a barrier and
    a device sync on both sides; returns the MAX elapsed seconds over ranks (the job's
    wall time).  `sync` is the device synchronisation (torch.cuda.synchronize on GPU)."""
    sync = sync or (lambda: None)
    for _ in range(warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


PEAK_HBM_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)


def kernel_breakdown(model, step, clips, streams, n_steps, split_desc=None):
    """Per-op table of the ViViT-B forward: `n_steps` extra (untimed) steps with HIP events
    around EVERY launch, on the stream each launch runs on; per op the mean launch duration,
    its share of the step and the achieved rate against the op's own roofline (MFMA for the
    GEMMs / attention in algorithmic FLOPs, HBM for LayerNorm / im2col in algorithmic bytes).
    `clips` = clips per launch (the mean over the parts when `split_desc` names uneven parts: the
    rates are then total work over total time)."""
    S, D, F, P = 3137, 768, 3072, 3136
    M = clips * S
    work = {  # (amount per launch, unit, bound)
        "im2col": (clips * (32 * 3 * 224 * 224 * 4 + P * 1536 * 2), "GB/s", "hbm"),
        "embed": (2.0 * clips * P * D * 1536, "TFLOP/s", "mfma"),
        "layernorm": (M * D * (4 + 2), "GB/s", "hbm"),
        "qkv": (2.0 * M * 3 * D * D, "TFLOP/s", "mfma"),
        "attention": (4.0 * S * S * 64 * 12 * clips, "TFLOP/s", "mfma"),
        "o_proj": (2.0 * M * D * D, "TFLOP/s", "mfma"),
        "fc1": (2.0 * M * F * D, "TFLOP/s", "mfma"),
        "fc2": (2.0 * M * D * F, "TFLOP/s", "mfma"),
    }
    ev = {}
    model.kernel_events = ev
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_steps):
        step()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / n_steps * 1e3
    model.kernel_events = None
    out = {}
    for name, (amt, unit, bound) in work.items():
        ms = [e0.elapsed_time(e1) for e0, e1 in ev.get(name, [])]
        if not ms:
            continue
        avg = float(np.mean(ms))
        rate = amt / (avg * 1e-3) / (1e12 if unit == "TFLOP/s" else 1e9)
        peak = PEAK_BF16_TFLOPS if bound == "mfma" else PEAK_HBM_GBS
        out[name] = {"launches_per_step": len(ms) // n_steps, "avg_launch_ms": round(avg, 4),
                     "share_of_step": round(sum(ms) / n_steps / step_ms, 4), "bound": bound,
                     "achieved": round(rate, 1), "unit": unit, "peak": peak, "frac": round(rate / peak, 4)}
    per = f"{split_desc} clips per launch, mean {clips:g}" if split_desc else f"{clips:g} clips per launch"
    out["note"] = (f"{n_steps} extra untimed steps with HIP events around every launch ({per}: "
                   f"the headline's {streams}-part split serialised on one stream); step {step_ms:.3f} ms under that "
                   "instrumentation; algorithmic work (M = clips x 3137 rows, no padding)")
    return out


def cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo), for the cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(model_cfg, n_clips, batch, gpu_logits_fns):
    """The fp32 CPU oracle (oracle/vivit_ref.py, a 'port' of the reference's HF ViViT forward) on
    the host cores, on bounded samples of the benchmark workload: `n_clips` clips
    one at a time (B=1, as the reference's inference CLI runs) and one batch of `batch` clips (the
    bench's own rank-0 batch, RandomState(1)).  The GPU logit errors (one per entry of
    `gpu_logits_fns`: the bf16 headline build and the fp16-operand build) are measured on that
    batch, i.e. on exactly the clips the timed region runs."""
    from oracle.vivit_ref import vivit_forward
    from vclip_amd.weights import make_synthetic_clips, make_vivit_weights

    sd = {k: torch.from_numpy(v) for k, v in make_vivit_weights(model_cfg, seed=0).items()}
    pix = make_synthetic_clips(batch, model_cfg["num_frames"], model_cfg["image_size"], seed=1)
    cores = torch.get_num_threads()
    with torch.no_grad():
        vivit_forward(sd, model_cfg, torch.from_numpy(pix[:1]))  # warm-up
        t0 = time.perf_counter()
        for i in range(n_clips):
            vivit_forward(sd, model_cfg, torch.from_numpy(pix[i:i + 1]))
        dt1 = time.perf_counter() - t0
        t0 = time.perf_counter()
        ref = vivit_forward(sd, model_cfg, torch.from_numpy(pix)).numpy()
        dtb = time.perf_counter() - t0
    err = {k: float(np.abs(fn(pix) - ref).max()) for k, fn in gpu_logits_fns.items()}
    return {"value": n_clips / dt1, "unit": "clips/s", "cores": cores, "kind": "port", "cpu": cpu_model(),
            "value_b8": round(batch / dtb, 4),
            "sample": f"ViViT-B/16x2 32x224^2 fp32 forward on the host: {n_clips} clips at B=1 (value) and one "
                      f"B={batch} batch (value_b8) of the bench's own clips, oracle/vivit_ref.py (eager attention), "
                      f"torch CPU {cores} threads"}, err


def cpu_lstm_cfg1():
    """BASELINE configs[0]: resnet50-2d-lstm forward, 8x224^2 clip, batch 1, on the CPU (the reference
    path; resnet50-2d-lstm/src/models/model.py:36-60 restated in oracle/lstm_ref.py, torch's nn.LSTM)."""
    from oracle.lstm_ref import lstm_forward
    from vclip_amd.weights import make_resnet50_lstm_weights, make_synthetic_video
    p = {k: torch.from_numpy(v) for k, v in make_resnet50_lstm_weights(seed=0).items()}
    x = torch.from_numpy(make_synthetic_video(1, 8, 224, seed=1))
    with torch.no_grad():
        lstm_forward(p, x)
        t0 = time.perf_counter()
        lstm_forward(p, x)
        dt = time.perf_counter() - t0
    return {"value": round(1.0 / dt, 4), "unit": "clips/s", "ms_per_clip": round(dt * 1e3, 1),
            "gflop_per_clip": 65.44, "cores": torch.get_num_threads(), "cpu": cpu_model(),
            "workload": "ResNet50-LSTM forward, 8x224x224 clip, batch 1, fp32 (BASELINE configs[0])"}


TRAIN_ATTN_GFLOP_PER_CLIP_LAYER = 2 * ATTN_GFLOP_PER_CLIP_LAYER  # dV, dP, dK, dQ (recompute of S not counted)
TRAIN_ATTN_BWD_KERNELS = ("abwd::attn_bwd_prep_kernel", "abwd::attn_bwd_dkdv_kernel", "abwd::attn_bwd_dq_kernel")


def cpu_train_baseline(n_clips):
    """The fp32 oracle's train step on the host cores (torch autograd + torch AdamW over the
    oracle/vivit_ref.py forward): a bounded sample of n_clips one-clip steps."""
    from oracle.vivit_ref import vivit_forward
    from vclip_amd.weights import make_synthetic_clips, make_vivit_weights
    cfg = dict(hidden_size=768, intermediate_size=3072, tubelet_size=[2, 16, 16], num_channels=3, num_frames=32,
               image_size=224, num_hidden_layers=12, num_labels=2, num_attention_heads=12, layer_norm_eps=1e-6)
    sd = {k: torch.from_numpy(v).requires_grad_() for k, v in make_vivit_weights(cfg, seed=0).items()}
    opt = torch.optim.AdamW(list(sd.values()), lr=1e-3, weight_decay=0.01)
    pix = torch.from_numpy(make_synthetic_clips(n_clips, 32, 224, seed=1))
    labels = torch.zeros(n_clips, dtype=torch.long)
    cores = torch.get_num_threads()
    t0 = time.perf_counter()
    for i in range(n_clips):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(vivit_forward(sd, cfg, pix[i:i + 1]), labels[i:i + 1]).backward()
        opt.step()
    dt = time.perf_counter() - t0
    return {"value": n_clips / dt, "unit": "clips/s", "cores": cores, "kind": "port",
            "sample": f"{n_clips} one-clip train steps (fwd + autograd bwd + torch AdamW) of the fp32 oracle "
                      f"(oracle/vivit_ref.py, eager attention), torch CPU {cores} threads"}


FAMILIES = {
    # mode: (metric, GFLOP per clip, default clips per GPU, BASELINE config, attention
    # kernel, its rocprofv3 name (the key of its counters in profiles/rNN_*_{traffic,pmc}.json))
    "timesformer": ("clips/sec fwd TimeSformer-B 8x224^2 bf16", 391.66, 16,
                    "TimeSformer-B divided space-time attention, 8x224x224 clips, batch 16 per GPU (BASELINE configs[2])",
                    "attn_short_d64_kernel (spatial branch: B*T sequences of 197 tokens, one 8-wave "
                    "workgroup per (sequence, head), all keys in LDS)",
                    "ashort::attn_short_d64_kernel<0, 7>"),
    "swin": ("clips/sec fwd Video Swin-T 32x224^2 bf16", 175.53, 4,
             "Video Swin-T 3D shifted-window attention, 32x224x224 clips, batch 4 per GPU = 32 over DP=8 "
             "(BASELINE configs[3])", "window_attn_mb_d32_kernel (all 12 blocks, head_dim 32; relative-position bias "
             "and shift mask on the matrix pipe)",
             "window_attn_mb_d32_kernel"),
    "resnet3d": ("clips/sec fwd ResNet3D-50 32x224^2 bf16", 349.0, 4,
                 "ResNet3D-50 (pytorchvideo create_resnet as resnet50-3d-video configures it), 32x224x224 clips, "
                 "batch 4 per GPU", None, None),
}

# rocprofv3 name prefixes of the non-GEMM kernels the recorder labels (ops.timed labels); GEMM labels
# are already rocprofv3 names (ops.GEMM_KERNEL)
PROF_NAME = {"attn_short_d64_kernel": "ashort::attn_short_d64_kernel<0, 7>",
             "window_attn_mb_d32_kernel": "window_attn_mb_d32_kernel",
             "attn_fwd_d64_kernel": ATTN_KERNEL}


def op_breakdown(model, step, n_steps: int):
    """`n_steps` extra (untimed) steps with HIP events around EVERY launch (ops.OpRecorder):
    per kernel instantiation its launches, mean launch time, share of the step and achieved rate on the
    algorithmic work the model states for it.  Returns (table sorted by share, step ms)."""
    from vclip_amd import ops
    with ops.recording(ops.OpRecorder()):
        step()  # discarded: one-time host work on the recorder's paths stays out of the table
    rec = ops.OpRecorder()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with ops.recording(rec):
        for _ in range(n_steps):
            step()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / n_steps * 1e3
    op_breakdown.last_ops = rec.summary_ops(n_steps, step_ms)
    return rec.summary(n_steps, step_ms), step_ms


# the fp16_precise leg's split-operand GEMMs (model.precise_ops): the embedding's weights and layer 0's
# q|k|v -- 6.3e-4 on 4 clips vs 6.7e-4 for the embedding's pixels and weights plus all of layer 0, at
# less than half its extra MFMA work (tests/test_fp16_gpu.py, round 5)
PRECISE_OPS = ("embed_w", "qkv")


def dominant_roofline(table, mode):
    """The roofline line of the kernel with the largest share of the step (op_breakdown's first row):
    GEMMs and attention against the bf16 MFMA peak, byte-moving kernels against HBM; traffic and PMC
    figures only from profiles/ of this build and mode."""
    kernel, row = next(iter(table.items()))
    mfma = row["unit"] == "TFLOP/s"
    peak = PEAK_BF16_TFLOPS if mfma else PEAK_HBM_GBS
    prof = PROF_NAME.get(kernel, kernel)
    traffic, traffic_src = measured_traffic(prof, mode)
    pmc, pmc_src = measured_pmc(prof, mode)
    mfma_busy, valu_per_mfma = pmc_rates(pmc)
    return {"bound": "mfma" if mfma else "hbm", "kernel": kernel, "ops": row["ops"], "achieved": row["achieved"],
            "peak": peak, "unit": row["unit"], "frac": round(row["achieved"] / peak, 4),
            "share_of_step": row["share_of_step"], "avg_launch_ms": row["avg_launch_ms"],
            "launches_per_step": row["launches_per_step"], "traffic": traffic, "traffic_source": traffic_src,
            "mfma_busy": mfma_busy, "valu_per_mfma": valu_per_mfma, "pmc_source": pmc_src,
            "timed_on": "HIP events around every launch of 3 extra steps of the headline's split, its parts "
                        "serialised on one stream (ops.OpRecorder); algorithmic work = real token rows and channels "
                        "(no padding)",
            "bound_rule": "per launch: HBM (algorithmic bytes: operands read once, the epilogue's output / residual "
                          "once) when its algorithmic flop per byte is below the 312.5 flop/B ridge (2.5 PFLOP/s bf16 "
                          "/ 8 TB/s), else the bf16 MFMA peak (ops.RIDGE_FLOP_PER_BYTE)"}


def cpu_family_baseline(mode, n_clips, gpu_logits_fn):
    """The family's fp32 CPU oracle (oracle/timesformer_ref.py, oracle/swin3d_ref.py) on the host
    cores, one clip at a time, plus the GPU logit error on the same clips."""
    from vclip_amd.weights import (make_swin3d_weights, make_synthetic_clips, make_synthetic_video,
                                   make_timesformer_weights)
    if mode == "timesformer":
        from oracle.timesformer_ref import timesformer_forward as fwd
        from vclip_amd.timesformer import TimesformerConfig
        c = TimesformerConfig(num_frames=8)
        cfg = dict(c.as_shape_cfg(), num_attention_heads=c.num_attention_heads, layer_norm_eps=c.layer_norm_eps,
                   hidden_act=c.hidden_act)
        sd = make_timesformer_weights(c.as_shape_cfg(), seed=0)
        x = make_synthetic_clips(n_clips, 8, 224, seed=1)
    elif mode == "swin":
        from oracle.swin3d_ref import swin3d_forward as fwd
        from vclip_amd.swin3d import SWIN3D_CONFIGS
        cfg = dict(SWIN3D_CONFIGS["tiny"], num_classes=2)
        sd = make_swin3d_weights(cfg, seed=0)
        x = make_synthetic_video(n_clips, 32, 224, seed=1)
    else:
        from oracle.resnet3d_ref import resnet3d_forward as fwd
        from vclip_amd.resnet3d import RESNET3D_50
        from vclip_amd.weights import make_resnet3d_weights
        cfg = dict(RESNET3D_50)
        sd = make_resnet3d_weights(cfg, seed=0)
        x = make_synthetic_video(n_clips, 32, 224, seed=1)
    sd = {k: torch.from_numpy(v) for k, v in sd.items()}
    cores = torch.get_num_threads()
    with torch.no_grad():
        fwd(sd, cfg, torch.from_numpy(x[:1]))  # warm-up
        t0 = time.perf_counter()
        ref = [fwd(sd, cfg, torch.from_numpy(x[i:i + 1])) for i in range(n_clips)]
        dt = time.perf_counter() - t0
    ref = torch.cat(ref).numpy()
    got = gpu_logits_fn(x)
    err = float(np.abs(got - ref).max())
    if mode == "resnet3d":  # random-init logits are O(5): the bar (tests/test_resnet3d_gpu.py) is relative
        err = err / max(1.0, float(np.abs(ref).max()))
    name = {"timesformer": "oracle/timesformer_ref.py", "swin": "oracle/swin3d_ref.py"}.get(mode, "oracle/resnet3d_ref.py")
    return {"value": n_clips / dt, "unit": "clips/s", "cores": cores, "kind": "port",
            "sample": f"{n_clips} clips fp32 forward, B=1 each, {name}, torch CPU {cores} threads"}, err


def run_family(a, dist, rank, world, dev):
    """BASELINE configs[2] / [3]: TimeSformer-B (divided space-time attention) and Video Swin-T
    (3D shifted windows) forwards, clips sharded per rank like the ViViT bench (no collective)."""
    from vclip_amd.weights import make_synthetic_clips, make_synthetic_video
    metric, gflop, _, workload, kname, kprof = FAMILIES[a.mode]
    if a.mode == "timesformer":
        from vclip_amd.timesformer import create_model
        model = create_model(num_frames=8, device=dev)
        x = torch.from_numpy(make_synthetic_clips(a.batch, 8, 224, seed=1 + rank)).to(dev)
    elif a.mode == "swin":
        from vclip_amd.swin3d import create_model
        model = create_model(model_size="tiny", device=dev)
        x = torch.from_numpy(make_synthetic_video(a.batch, 32, 224, seed=1 + rank)).to(dev)
    else:
        from vclip_amd.resnet3d import create_model
        model = create_model(device=dev).eval()
        x = torch.from_numpy(make_synthetic_video(a.batch, 32, 224, seed=1 + rank)).to(dev)

    model.graph_replay = bool(a.graph)

    def step():
        model.forward_logits(x)

    def timed(streams):
        model.concurrent_streams = streams
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        return timed_loop(step, a.steps, 0, dist, torch.cuda.synchronize)

    # headline: the batch over `--streams` HIP streams (graph replay), nothing instrumented; then the
    # per-kernel table of 3 one-stream steps with HIP events around every launch, whose largest row is
    # the roofline line (the step's dominant kernel)
    dt = timed(a.streams)
    tune = _stream_tuning(model)
    model.graph_replay = False  # the passes below are event-instrumented or one-off calls
    dt1 = timed(1)
    # the per-kernel table on the headline's own launches: its split, the parts serialised on one stream
    model.concurrent_streams = a.streams
    with vstreams.serial_parts():
        table, instr_ms = op_breakdown(model, step, 3)
    model.concurrent_streams = 1
    value = a.batch * a.steps * world / dt
    ms_per_step = dt / a.steps * 1e3
    model_tflops = gflop * a.batch / (ms_per_step * 1e-3) / 1e3
    out = None
    if rank == 0:
        roof = dominant_roofline(table, a.mode)
        roof["one_stream_clips_s"] = round(a.batch * a.steps * world / dt1, 2)
        attn = None
        if kprof is not None:
            # the family's attention kernel beside it: intensity N / 2 flop per byte (N keys per
            # sequence | window; q, k, v read and the output written once, 8 B per token x head-dim
            # element) puts it below the 312 flop/B ridge, so HBM is its algorithmic bound
            akey = next(k for k in table if k in PROF_NAME and PROF_NAME[k] == kprof)
            arow = table[akey]
            unit_n = 197 if a.mode == "timesformer" else 392
            gbs = arow["achieved"] * 1e3 / (unit_n / 2)
            traffic, traffic_src = measured_traffic(kprof, a.mode)
            pmc, pmc_src = measured_pmc(kprof, a.mode)
            mfma_busy, valu_per_mfma = pmc_rates(pmc)
            attn = {"kernel": kname, "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(gbs / PEAK_HBM_GBS, 4), "achieved_tflops": arow["achieved"],
                    "mfma_frac": round(arow["achieved"] / PEAK_BF16_TFLOPS, 4), "share_of_step": arow["share_of_step"],
                    "avg_launch_ms": arow["avg_launch_ms"], "intensity_flop_per_byte": unit_n / 2,
                    "traffic": traffic, "traffic_source": traffic_src, "mfma_busy": mfma_busy,
                    "valu_per_mfma": valu_per_mfma, "pmc_source": pmc_src,
                    "executed_work_note": ("window_attn_mb_d32_kernel issues 2 identity-bias MFMAs (+1 mask MFMA in "
                                           "shifted windows) per 32-key block beside the 2 QK^T MFMAs and streams its "
                                           "fp16 bias operand from L2: executed MFMA work ~2x the algorithmic flops "
                                           "counted here" if a.mode == "swin" else None)}
        cpu, err = None, None
        if world == 1 and not a.no_cpu_baseline:
            cpu, err = cpu_family_baseline(
                a.mode, a.cpu_clips, lambda p: model.forward_logits(torch.from_numpy(p).to(dev)).cpu().numpy().copy())
        out = {
            "metric": metric, "value": round(value, 2), "unit": "clips/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (uint8 frames RandomState(1+rank) -> the family's processor affine; weights RandomState(0))",
            "config": {"workload": workload, "global_batch": a.batch * world, "parallelism": f"dp{world}",
                       "streams": a.streams, "hip_graph": _graph_used(model, a), "stream_sets_timed": tune},
            "logit_max_abs_err": err,
            "logit_err_note": "max |logit - oracle| relative to max(1, max |oracle logit|)" if a.mode == "resnet3d" else None,
            "roofline": roof,
            "attention_roofline": attn,
            "kernel_breakdown": dict(list(table.items())[:12], note=f"3 steps of the headline's {a.streams}-part split "
                                     "serialised on one stream, HIP events around every launch: "
                                     f"{instr_ms:.3f} ms per step under that instrumentation"),
            "op_breakdown": dict(list(op_breakdown.last_ops.items())[:24]),
            "model_tflops": round(model_tflops, 1), "model_frac_of_peak": round(model_tflops / PEAK_BF16_TFLOPS, 4),
            "cpu_baseline": cpu,
            "build": _build_id(),
        }
        print(json.dumps(out), flush=True)
    return out


WGRAD_KERNELS = ("trn::wgrad_pp_kernel", "trn::wgrad_big_kernel")


def wgrad_line(ktable, instr_ms):
    """the weight-gradient row of the train step's per-kernel table against the bf16 peak, with the
    weight-gradient kernel's counters of this build's train profile (when present)"""
    kern = next((k for k in WGRAD_KERNELS if f"{k} (+ wgrad_reduce_kernel)" in ktable), None)
    if kern is None:
        return None
    label = f"{kern} (+ wgrad_reduce_kernel)"
    row = ktable[label]
    traffic, traffic_src = measured_traffic([kern, "trn::wgrad_reduce_kernel"], "train")
    pmc, pmc_src = measured_pmc(kern, "train")
    mfma_busy, valu_per_mfma = pmc_rates(pmc)
    return {"bound": "mfma", "kernel": label, "achieved": row["achieved"], "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s", "frac": round(row["achieved"] / PEAK_BF16_TFLOPS, 4),
            "avg_launch_ms": row["avg_launch_ms"], "launches_per_step": row["launches_per_step"],
            "share_of_step": row["share_of_step"], "traffic": traffic, "traffic_source": traffic_src,
            "mfma_busy": mfma_busy, "valu_per_mfma": valu_per_mfma, "pmc_source": pmc_src,
            "timed_on": f"2 extra steps, weight gradients on the chain's stream (the timed step runs them on a side "
                        f"stream), HIP events around each vc_wgrad_bf16 call: {instr_ms:.3f} ms per step there; work "
                        "2 M N1 N2 per call (M = the rows the call reduces over: the padded rows of the activations, 12800 at B = 4 for 12548 tokens)"}


def run_train(a, dist, rank, world, dev):
    """BASELINE configs[4]: the reference's train step (trainers/trainer.py:140-146) on the HIP
    model: zero_grad, forward, CrossEntropyLoss, backward (+ RCCL all-reduce for N > 1), AdamW."""
    from vclip_amd.dp import GradAllReduce
    from vclip_amd.optim import AdamW
    from vclip_amd.vivit import create_model
    from vclip_amd.weights import make_synthetic_clips

    model = create_model(num_frames=32, device=dev).train()
    opt = AdamW(model.parameters(), lr=1e-3, weight_decay=0.01)
    sync = GradAllReduce(model) if dist else None
    pix = torch.from_numpy(make_synthetic_clips(a.batch, 32, 224, seed=1 + rank)).to(dev)
    labels = torch.from_numpy(np.random.RandomState(2 + rank).randint(0, 2, size=a.batch)).long().to(dev)
    crit = torch.nn.CrossEntropyLoss()
    losses = []

    def step():
        opt.zero_grad()
        outputs = model(pixel_values=pix)
        loss = crit(outputs.logits, labels)
        loss.backward()
        if sync:
            sync.wait()
        opt.step()
        losses.append(loss.detach())

    # --train-graph 1 at world size 1: the whole step (forward, loss, backward, AdamW) captured once into a
    # hipGraph and replayed (vivit_train.GraphedTrainStep: the same kernels in the same order, bit-identical to
    # the eager step).  Off by default: at B = 4 the eager step is not launch-bound and the replay measured
    # 2 % slower (212.3 vs 216.6 clips/s, round 6)
    graphed = bool(a.train_graph) and not dist
    if graphed:
        from vclip_amd.vivit_train import GraphedTrainStep
        gstep = GraphedTrainStep(model, opt, crit, pix, labels, warmup=max(2, a.warmup))

        def timed_step():
            losses.append(gstep().detach().clone())
    else:
        timed_step = step
        for _ in range(a.warmup):
            step()
    torch.cuda.synchronize()
    dt = timed_loop(timed_step, a.steps, 1 if graphed else 0, dist, torch.cuda.synchronize)
    # the attention backward's roofline: HIP events around each of its launches in 2 extra eager steps (an
    # event inside a replayed graph would be frozen at capture)
    evs = []
    model._engine.kernel_events = evs
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    model._engine.kernel_events = None
    attn_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    # the step's largest kernel by GPU time, the weight gradients (vc_wgrad_bf16: trn::wgrad_big_kernel +
    # its split-K reduction): 2 extra steps with HIP events around every GEMM / weight-gradient launch, the
    # weight gradients on the chain's own stream for that pass (side_wgrad off) so each event times its
    # launch alone
    from vclip_amd import ops
    eng = model._engine
    side = eng.side_wgrad
    eng.side_wgrad = False
    rec = ops.OpRecorder()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with ops.recording(rec):
        for _ in range(2):
            step()
    torch.cuda.synchronize()
    instr_ms = (time.perf_counter() - t0) / 2 * 1e3
    eng.side_wgrad = side
    ktable = rec.summary(2, instr_ms)
    clips = a.batch * a.steps * world
    value = clips / dt
    ms_per_step = dt / a.steps * 1e3
    attn_tflops = TRAIN_ATTN_GFLOP_PER_CLIP_LAYER * a.batch / (attn_ms * 1e-3) / 1e3
    step_tflops = 3 * VIVIT_GFLOP_PER_CLIP * a.batch / (ms_per_step * 1e-3) / 1e3
    out = None
    if rank == 0:
        # the roofline "launch" is one layer's attention backward: prep + dK/dV + dQ
        traffic, traffic_src = measured_traffic(TRAIN_ATTN_BWD_KERNELS, "train")
        pmc, pmc_src = measured_pmc(TRAIN_ATTN_BWD_KERNELS[1], "train")
        mfma_busy, valu_per_mfma = pmc_rates(pmc)
        cpu = None if (world > 1 or a.no_cpu_baseline) else cpu_train_baseline(a.cpu_clips)
        out = {
            "metric": "clips/sec train step (fwd+bwd+AdamW) ViViT-B 32x224^2 bf16",
            "value": round(value, 2), "unit": "clips/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uint8 frames RandomState(1+rank) -> ViViT processor affine, labels RandomState(2+rank); "
                    "weights RandomState(0))",
            "config": {"workload": f"ViViT-B/16x2 train step, 32x224x224 clips, batch {a.batch} per GPU, AdamW(lr 1e-3, "
                                   "wd 0.01), RCCL gradient all-reduce for N > 1 (BASELINE configs[4])",
                       "model": "ViViT-B/16x2 (joint space-time, 12L, d768, 12H, 3137 tokens)",
                       "global_batch": a.batch * world, "seq_len": 3137, "parallelism": f"dp{world}",
                       "hip_graph": graphed},
            "loss_first_last": [round(float(losses[0]), 5), round(float(losses[-1]), 5)],
            "roofline": {"bound": "mfma", "kernel": "attention backward (attn_bwd_dkdv + attn_bwd_dq + prep)",
                         "achieved": round(attn_tflops, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(attn_tflops / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "algorithmic_bytes": TRAIN_ATTN_IO_BYTES_PER_CLIP * a.batch,
                         "avg_launch_ms": round(attn_ms, 4), "mfma_busy_dkdv": mfma_busy, "valu_per_mfma_dkdv": valu_per_mfma, "pmc_source": pmc_src,
                         "flop_per_launch": f"{TRAIN_ATTN_GFLOP_PER_CLIP_LAYER:.2f} GF/clip x {a.batch} clips"},
            "step_tflops": round(step_tflops, 1), "step_frac_of_peak": round(step_tflops / PEAK_BF16_TFLOPS, 4),
            "wgrad_roofline": wgrad_line(ktable, instr_ms),
            "kernel_table": dict(list(ktable.items())[:10], note="2 extra steps, weight gradients on the chain's "
                                 "stream, HIP events around every GEMM / weight-gradient launch (ops.OpRecorder): "
                                 f"{instr_ms:.3f} ms per step under that instrumentation; the attention backward "
                                 "is timed separately (roofline)"),
            "cpu_baseline": cpu,
            "build": _build_id(),
        }
        print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["fwd", "train", "timesformer", "swin", "resnet3d"], default="fwd")
    ap.add_argument("--batch", type=int, default=None, help="clips per GPU per step (fwd 8, train 4)")
    ap.add_argument("--cpu-clips", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=None,
                    help="inference modes: concurrent HIP streams the batch is split over in the headline pass "
                         "(default 2; swin 4: its late stages' short launches, measured under graph replay)")
    ap.add_argument("--graph", type=int, default=1,
                    help="inference modes: 1 = the headline forward replayed from its captured hipGraph "
                         "(model.graph_replay; the event-instrumented roofline passes stay eager), 0 = eager; "
                         "train: see --train-graph")
    ap.add_argument("--train-graph", type=int, default=0,
                    help="train at world size 1: 1 = the whole step captured once into a hipGraph and replayed "
                         "(vivit_train.GraphedTrainStep), 0 = the eager step (default)")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)  # CPU test of the spawn path
    a = ap.parse_args()
    if a.streams is None:
        a.streams = 4 if a.mode == "swin" else 2
    if a.batch is None:
        a.batch = {"fwd": 8, "train": 4}.get(a.mode) or FAMILIES[a.mode][2]
    if a.cpu_clips is None:
        a.cpu_clips = {"fwd": 2, "timesformer": 3, "resnet3d": 2}.get(a.mode, 1)

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(_spawn_world(a.gpus))
    if int(os.environ.get("WORLD_SIZE", "1")) != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')} "
                         "(launch N ranks, or pass --gpus N without a launcher to spawn them)")
    if a.launch_check:  # tests/test_dist_cpu.py: ranks rendezvous over gloo, no GPU touched
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dt = timed_loop(lambda: None, a.steps, a.warmup, tdist)
        if tdist.get_rank() == 0:
            print(json.dumps({"n_gpus": tdist.get_world_size(), "world_size_env": int(os.environ["WORLD_SIZE"]),
                              "steps": a.steps, "seconds": dt}), flush=True)
        tdist.barrier()
        tdist.destroy_process_group()
        return None
    dist, rank, world, local = _dist()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if a.mode in FAMILIES:
        out = run_family(a, dist, rank, world, dev)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return out
    if a.mode == "train":
        out = run_train(a, dist, rank, world, dev)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return out

    from vclip_amd.vivit import create_model
    from vclip_amd.weights import make_synthetic_clips

    model = create_model(num_frames=32, device=dev)
    cfg = model.config
    pix = torch.from_numpy(make_synthetic_clips(a.batch, 32, 224, seed=1 + rank)).to(dev)

    model.graph_replay = bool(a.graph)

    def step():
        model.forward_logits(pix)

    def timed(streams, evs=None):
        """W warm-up + K timed steps with the batch on `streams` concurrent HIP streams; `evs`: a list
        that collects HIP events around every attention launch (on the stream it runs on)."""
        model.concurrent_streams = streams
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        model.kernel_events = evs
        t = timed_loop(step, a.steps, 0, dist, torch.cuda.synchronize)
        model.kernel_events = None
        return t

    # the headline: the batch split over `--streams` concurrent HIP streams (the clips are independent,
    # every kernel is batch-invariant: logits bit-identical to one stream), nothing instrumented
    dt = timed(a.streams)
    tune = _stream_tuning(model)
    streams = model.last_streams
    split = list(model.last_split)  # clips per part (vivit.SPLIT_DEFAULT: 5 + 3 at B = 8 on two streams)
    split_desc = " + ".join(str(v) for v in split)
    graphed = model.graph_replay
    # the fp16-operand build of the same forward (VC_ELEM_F16: same kernels, same MFMA rate, logits
    # within 1e-3) and its split-operand variant (precise_layers = 1 with PRECISE_OPS: the weights of
    # the first layers set the fp16 build's logit error), each timed like the headline
    # beside a bf16 re-run, alternating bf16 / fp16 / fp16_precise twice: the chip's clock drifts over a
    # run, so legs timed once after the instrumented passes read low against the opening headline
    legs = {"bf16": [], "fp16": [], "fp16_precise": []}
    for _ in range(2):
        for leg in legs:
            model.compute_dtype = torch.bfloat16 if leg == "bf16" else torch.float16
            model.precise_layers = 1 if leg == "fp16_precise" else 0
            model.precise_ops = PRECISE_OPS
            model.graph_replay = graphed
            legs[leg].append(timed(a.streams))
    model.graph_replay = graphed
    model.precise_layers = 0
    model.compute_dtype = torch.bfloat16
    dt16, dt16p, dtb = float(np.median(legs["fp16"])), float(np.median(legs["fp16_precise"])), float(np.median(legs["bf16"]))
    model.graph_replay = False  # the event-instrumented passes and one-off calls below run eagerly
    # the kernel roofline on the headline's OWN launches: the same split (batch / streams clips per launch,
    # the same kernels and workspaces) with the parts one after the other on one stream and HIP events
    # around every attention launch, so a launch's event time is its own execution (under two concurrent
    # streams it would include time shared with the other part's kernels); rocprofv3 of
    # `tools/headline.py --serial 1` times the same launches (tools/profile_round.sh)
    evs = []
    with vstreams.serial_parts():
        dts = timed(a.streams, evs)
    attn_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    # ... and the whole batch as ONE launch per op on one stream (round-4's roofline pass), for reference
    evs1 = []
    dt1 = timed(1, evs1)
    attn_ms1 = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs1]))
    # the fp16 build's attention launches, timed like the bf16 roofline pass
    model.compute_dtype = torch.float16
    evs16 = []
    with vstreams.serial_parts():
        timed(a.streams, evs16)
    attn_ms16 = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs16]))
    model.compute_dtype = torch.bfloat16
    # per-op and per-kernel tables of the headline's own launches (its split, serialised on one stream)
    model.concurrent_streams = streams
    part_clips = a.batch // streams if a.batch % streams == 0 else a.batch / streams
    with vstreams.serial_parts():
        breakdown = kernel_breakdown(model, step, part_clips, streams, 3, split_desc)
        ktable, instr_ms = op_breakdown(model, step, 3)
    model.concurrent_streams = 1

    clips = a.batch * a.steps * world
    value = clips / dt
    ms_per_step = dt / a.steps * 1e3
    # the roofline pass times the headline's launches: `split` clips each, mean batch / streams (mean rate =
    # total attention work over total launch time)
    launch_clips = part_clips
    attn_tflops = ATTN_GFLOP_PER_CLIP_LAYER * launch_clips / (attn_ms * 1e-3) / 1e3
    attn_tflops1 = ATTN_GFLOP_PER_CLIP_LAYER * a.batch / (attn_ms1 * 1e-3) / 1e3
    model_tflops = VIVIT_GFLOP_PER_CLIP * a.batch / (ms_per_step * 1e-3) / 1e3

    out = None
    if rank == 0:
        cpu = None
        logit_err = logit_err16 = logit_err16p = None
        traffic, traffic_src = measured_traffic(ATTN_KERNEL, "fwd")
        pmc, pmc_src = measured_pmc(ATTN_KERNEL, "fwd")
        mfma_busy, valu_per_mfma = pmc_rates(pmc)
        if world == 1 and not a.no_cpu_baseline:
            shape_cfg = dict(cfg.as_shape_cfg(), num_attention_heads=cfg.num_attention_heads,
                             layer_norm_eps=cfg.layer_norm_eps)

            def gpu_logits(dtype, precise=0):
                def fn(p):
                    model.compute_dtype = dtype
                    model.precise_layers = precise
                    model.precise_ops = PRECISE_OPS
                    lg = model.forward_logits(torch.from_numpy(p).to(dev)).cpu().numpy().copy()
                    model.compute_dtype = torch.bfloat16
                    model.precise_layers = 0
                    return lg
                return fn

            cpu, errs = cpu_baseline(shape_cfg, a.cpu_clips, a.batch,
                                     {"bf16": gpu_logits(torch.bfloat16), "fp16": gpu_logits(torch.float16),
                                      "fp16_precise": gpu_logits(torch.float16, 1)})
            logit_err, logit_err16, logit_err16p = errs["bf16"], errs["fp16"], errs["fp16_precise"]
            cpu["lstm_cfg1"] = cpu_lstm_cfg1()
        out = {
            "metric": "clips/sec fwd ViViT-B 32x224^2 bf16",
            "value": round(value, 2),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uint8 frames RandomState(1+rank) -> ViViT processor affine; weights RandomState(0))",
            "config": {"workload": "ViViT-B/16x2 forward, 32x224x224 clips, batch 8 per GPU (BASELINE configs[1])",
                       "model": "ViViT-B/16x2 (joint space-time, 12L, d768, 12H, 3137 tokens)",
                       "global_batch": a.batch * world, "seq_len": 3137, "parallelism": f"dp{world}",
                       "streams": a.streams, "split": split, "hip_graph": _graph_used(model, a),
                       "stream_sets_timed": tune},
            "logit_max_abs_err": logit_err,
            "roofline": {"bound": "mfma", "kernel": ATTN_KERNEL, "achieved": round(attn_tflops, 1),
                         "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(attn_tflops / PEAK_BF16_TFLOPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes": ATTN_IO_BYTES_PER_CLIP * launch_clips, "avg_launch_ms": round(attn_ms, 4),
                         "flop_per_launch": f"{ATTN_GFLOP_PER_CLIP_LAYER:.2f} GF/clip x {launch_clips:g} clips (mean of "
                                            f"the {split_desc}-clip launches)",
                         "timed_on": f"the headline's own launches ({split_desc} clips: its {streams}-stream "
                                     "split) run one after the other on one HIP stream, HIP events around every "
                                     f"attention launch: clips/s {a.batch * a.steps * world / dts:.2f} there",
                         "whole_batch_launch": {"clips": a.batch, "avg_launch_ms": round(attn_ms1, 4),
                                                "achieved": round(attn_tflops1, 1),
                                                "frac": round(attn_tflops1 / PEAK_BF16_TFLOPS, 4),
                                                "one_stream_clips_s": round(a.batch * a.steps * world / dt1, 2)},
                         "mfma_busy": mfma_busy, "valu_per_mfma": valu_per_mfma,
                         "pmc_source": pmc_src},
            "kernel_breakdown": breakdown,
            "kernel_table": dict(ktable, note=f"per kernel instantiation (ops.OpRecorder), 3 steps of the headline's "
                                 f"{streams}-part split serialised on one stream, HIP events around every launch: "
                                 f"{instr_ms:.3f} ms per step under that instrumentation"),
            "build": _build_id(),
            "model_tflops": round(model_tflops, 1),
            "model_frac_of_peak": round(model_tflops / PEAK_BF16_TFLOPS, 4),
            "fp16": {"value": round(clips / dt16, 2), "ms_per_step": round(dt16 / a.steps * 1e3, 3),
                     "vs_bf16_same_conditions": round(dtb / dt16, 4),
                     "logit_max_abs_err": logit_err16, "attn_avg_launch_ms": round(attn_ms16, 4),
                     "attn_frac": round(ATTN_GFLOP_PER_CLIP_LAYER * launch_clips / (attn_ms16 * 1e-3) / 1e3
                                        / PEAK_BF16_TFLOPS, 4),
                     "note": "same forward with fp16 MFMA operands (VC_ELEM_F16; fp16 dense peak = bf16's); median "
                             "of 2 runs alternating with bf16 re-runs (bf16_same_conditions); its gap to bf16 is the "
                             "clock: same shader cycles, -2.7 % effective clock under fp16 operand data "
                             "(profiles/r05_fp16_clock.json)"},
            "fp16_precise": {"value": round(clips / dt16p, 2), "ms_per_step": round(dt16p / a.steps * 1e3, 3),
                             "vs_bf16_same_conditions": round(dtb / dt16p, 4),
                             "logit_max_abs_err": logit_err16p, "precise_ops": list(PRECISE_OPS),
                             "note": "fp16 build with split operands (fp16 high + low parts: vc_gemm_h16_wrap) in the "
                                     "patch embedding's weights and layer 0's q|k|v GEMM (model.precise_layers = 1, "
                                     "model.precise_ops)"},
            "bf16_same_conditions": {"value": round(clips / dtb, 2), "note": "bf16 re-runs alternating with the fp16 "
                                     "legs (median of 2); the headline value is the first, opening run"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
