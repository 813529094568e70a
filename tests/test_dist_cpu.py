"""Multi-process (gloo, world_size 2) checks of the data-parallel bench path on CPU:
clips shard per rank with no data-path collective; the timed region is bracketed by
barriers and the reported wall time is the MAX over ranks."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    # rank r's step takes (r+1) * 20 ms: the job time is the slowest rank's
    def step():
        time.sleep(0.02 * (rank + 1))

    dt = bench.timed_loop(step, steps=5, warmup=1, dist=dist)
    # each rank shards its own clips: no collective inside the step; the logits of a rank's
    # shard depend only on its own inputs (seeded by rank, as bench.py does)
    from vclip_amd.weights import make_synthetic_clips
    x = make_synthetic_clips(2, 4, 32, seed=1 + rank)
    q.put((rank, dt, float(x.sum())))
    dist.barrier()
    dist.destroy_process_group()


def test_timed_loop_max_over_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    dts = [r[1] for r in res]
    assert abs(dts[0] - dts[1]) < 1e-9  # every rank reports the same (max) time
    assert dts[0] >= 5 * 0.04 * 0.95  # >= the slowest rank's 5 steps
    assert res[0][2] != res[1][2]  # ranks draw different clips


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus N` without a launcher starts N ranks itself (torch.distributed.run on
    127.0.0.1); a WORLD_SIZE that disagrees with --gpus is an error, not a silent 1-GPU run."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--launch-check"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["world_size_env"] == 2
    bad = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launch-check"],
                         capture_output=True, text=True, timeout=120, env=dict(env, WORLD_SIZE="1"))
    assert bad.returncode != 0 and "WORLD_SIZE" in (bad.stderr + bad.stdout)
