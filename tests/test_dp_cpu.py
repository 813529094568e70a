"""Data-parallel gradient exchange of the ViViT train step (BASELINE config 5)
on CPU with gloo, world_size 2: vclip_amd.dp.GradAllReduce driven by the same per-stage
`grad_ready_hooks` calls the HIP backward makes, over the model's real flat layout.

Checked: (1) buckets are contiguous, in backward-completion order, cover the whole flat
buffer and respect the bucket size; (2) the averaged per-rank gradients of each rank's
shard (fp32 oracle autograd, oracle/vivit_ref.py) equal the single-process gradient of the
concatenated batch — the property data-parallel training relies on.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

TINY = dict(image_size=32, num_frames=4, tubelet_size=[2, 16, 16], num_channels=3, hidden_size=256,
            num_hidden_layers=2, num_attention_heads=4, intermediate_size=512, hidden_act="gelu_fast",
            layer_norm_eps=1e-6, qkv_bias=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeModel:
    """Carries what GradAllReduce needs from VivitForVideoClassification: the hook list."""

    def __init__(self):
        self.grad_ready_hooks = []


def _flat_grads(layout, grads):
    flat = torch.zeros(layout.total)
    for n, g in grads.items():
        layout.view(flat, n).copy_(g.reshape(layout.entries[n][2]))
    return flat


def _shard_grads(sd, pix, labels):
    from oracle.vivit_ref import vivit_forward
    ref = {k: torch.from_numpy(v).clone().requires_grad_() for k, v in sd.items()}
    loss = torch.nn.functional.cross_entropy(vivit_forward(ref, TINY, pix), labels)
    loss.backward()
    return {k: v.grad for k, v in ref.items()}


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from vclip_amd.dp import GradAllReduce
    from vclip_amd.vivit import VivitConfig
    from vclip_amd.vivit_train import FlatLayout
    from vclip_amd.weights import make_synthetic_clips, make_vivit_weights, vivit_param_shapes

    cfg = VivitConfig(**TINY)
    layout = FlatLayout(cfg, vivit_param_shapes(cfg.as_shape_cfg()))
    sd = make_vivit_weights(TINY, seed=0)
    B = 2  # clips per rank
    pix = torch.from_numpy(make_synthetic_clips(B * world, 4, 32, seed=1))
    labels = torch.from_numpy(np.random.RandomState(2).randint(0, 2, size=B * world)).long()
    shard = slice(rank * B, (rank + 1) * B)
    gflat = _flat_grads(layout, _shard_grads(sd, pix[shard], labels[shard]))

    model = _FakeModel()
    sync = GradAllReduce(model, bucket_bytes=64 * 1024)
    for stage, start, end in layout.stages:  # the order the HIP backward reports them
        for h in model.grad_ready_hooks:
            h(stage, start, end, gflat)
    launched = sync.wait()
    q.put((rank, gflat.numpy(), launched, layout.total))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_gloo_matches_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, g0, launched, total), (_, g1, _, _) = res
    np.testing.assert_array_equal(g0, g1)  # every rank holds the same averaged gradient
    # buckets: contiguous, in order, covering [0, total); each closed once it reached 64 KiB
    assert launched[0][0] == 0 and launched[-1][1] == total
    for (a, b), (c, d) in zip(launched, launched[1:]):
        assert b == c
    assert all(b - a >= 16 * 1024 for a, b in launched[:-1])
    # == the gradient of the mean loss over the concatenated batch (one process)
    from vclip_amd.vivit import VivitConfig
    from vclip_amd.vivit_train import FlatLayout
    from vclip_amd.weights import make_synthetic_clips, make_vivit_weights, vivit_param_shapes
    cfg = VivitConfig(**TINY)
    layout = FlatLayout(cfg, vivit_param_shapes(cfg.as_shape_cfg()))
    sd = make_vivit_weights(TINY, seed=0)
    pix = torch.from_numpy(make_synthetic_clips(2 * world, 4, 32, seed=1))
    labels = torch.from_numpy(np.random.RandomState(2).randint(0, 2, size=2 * world)).long()
    full = _flat_grads(layout, _shard_grads(sd, pix, labels)).numpy()
    np.testing.assert_allclose(g0, full, rtol=1e-4, atol=1e-7)
