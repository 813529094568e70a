"""GradAllReduce on the GPU through the real model backward:
an RCCL (nccl backend) world of one rank drives the side-stream branch of dp.py -- the event wait,
all_reduce(ReduceOp.AVG, async_op=True).wait() on the side stream, the join in wait() -- from the
hooks VivitForVideoClassification's backward fires.  With one rank the average is the identity, so
the gradient the optimizer sees must equal the un-synchronised backward's bit for bit; the buckets
must tile the flat gradient buffer, also when gradients accumulate over two backwards."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = dict(image_size=32, num_frames=4, tubelet_size=[2, 16, 16], num_channels=3, hidden_size=256,
           num_hidden_layers=2, num_attention_heads=4, intermediate_size=512, hidden_act="gelu_fast",
           layer_norm_eps=1e-6, qkv_bias=True)


@pytest.fixture(scope="module")
def rccl():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def _model_and_batch(B=2):
    from vclip_amd.vivit import VivitConfig, VivitForVideoClassification
    from vclip_amd.weights import make_synthetic_clips, make_vivit_weights
    model = VivitForVideoClassification(VivitConfig(**CFG, id2label={0: "a", 1: "b"}))
    model.load_state_dict(make_vivit_weights(CFG, seed=0))
    model = model.to("cuda").train()
    pix = torch.from_numpy(make_synthetic_clips(B, 4, 32, seed=1)).cuda()
    labels = torch.tensor([0, 1][:B], device="cuda")
    return model, pix, labels


def _grads(model):
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def _step(model, pix, labels):
    loss = torch.nn.functional.cross_entropy(model(pixel_values=pix).logits, labels)
    loss.backward()


def test_grad_allreduce_rccl_side_stream(rccl):
    from vclip_amd.dp import GradAllReduce
    model, pix, labels = _model_and_batch()
    model.zero_grad(set_to_none=True)
    _step(model, pix, labels)
    ref = _grads(model)
    model.zero_grad(set_to_none=True)
    sync = GradAllReduce(model, bucket_bytes=1 << 20)  # small buckets: several launches
    _step(model, pix, labels)
    launched = sync.wait()
    assert sync._side is not None  # the CUDA side-stream branch ran
    assert len(launched) > 1
    total = model._gflat.numel()
    spans = sorted(launched)
    assert spans[0][0] == 0 and spans[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))  # contiguous, no gap / overlap
    got = _grads(model)
    for n in ref:
        assert torch.equal(got[n], ref[n]), n


def test_grad_allreduce_with_accumulation(rccl):
    """Two backwards without zero_grad: the hooks fire on the accumulated buffer (ADVICE r1:
    they used to be skipped, leaving ranks on local gradients)."""
    from vclip_amd.dp import GradAllReduce
    model, pix, labels = _model_and_batch()
    model.zero_grad(set_to_none=True)
    _step(model, pix, labels)
    _step(model, pix, labels)
    ref = _grads(model)
    model.zero_grad(set_to_none=True)
    sync = GradAllReduce(model)
    _step(model, pix, labels)
    first = sync.wait()
    _step(model, pix, labels)
    second = sync.wait()
    total = model._gflat.numel()
    for launched in (first, second):
        spans = sorted(launched)
        assert spans[0][0] == 0 and spans[-1][1] == total
    got = _grads(model)
    for n in ref:
        torch.testing.assert_close(got[n], ref[n], rtol=0, atol=0)


def test_optimizer_subset_is_not_flat(rccl):
    """AdamW over a parameter subset must not update the rest of the flat buffer."""
    from vclip_amd.optim import AdamW
    model, pix, labels = _model_and_batch()
    head = [p for n, p in model.named_parameters() if "classifier" in n]
    opt = AdamW(head, lr=1e-2, weight_decay=0.01)
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    model.zero_grad(set_to_none=True)
    _step(model, pix, labels)
    opt.step()
    for n, p in model.named_parameters():
        changed = not torch.equal(p.detach(), before[n])
        assert changed == ("classifier" in n), n
    np.testing.assert_equal(len(opt.state), 2)


def test_optimizer_full_layout_is_one_launch(rccl):
    """AdamW over every parameter of the ViViT flat layout takes the one-launch path (its alignment
    gaps stay zero) and matches torch.optim.AdamW on the same gradients."""
    from vclip_amd.optim import AdamW
    model, pix, labels = _model_and_batch()
    opt = AdamW(model.parameters(), lr=1e-3, weight_decay=0.01)
    model.zero_grad(set_to_none=True)
    _step(model, pix, labels)
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    grads = _grads(model)
    opt.step()
    assert "flat" in opt.state and len(opt.state) == 1
    ref = {n: torch.nn.Parameter(before[n].clone()) for n in before}
    for n, q in ref.items():
        q.grad = grads[n].clone()
    torch.optim.AdamW(list(ref.values()), lr=1e-3, weight_decay=0.01).step()
    for n, p in model.named_parameters():
        torch.testing.assert_close(p.detach(), ref[n].detach(), rtol=1e-6, atol=1e-7)
    flat = model._flat
    gaps = torch.ones(flat.numel(), dtype=torch.bool, device=flat.device)
    for p in model.parameters():
        gaps[p.storage_offset():p.storage_offset() + p.numel()] = False
    assert torch.count_nonzero(flat[gaps]) == 0  # the layout's alignment gaps stay zero


def test_graph_capture_under_live_rccl_group(rccl):
    """bench.py --gpus N > 1 captures each rank's forward into a hipGraph while its RCCL process
    group is up (capture_error_mode="thread_local": the group's watchdog thread keeps making HIP
    calls).  Here, after a collective has run on the group, the ViViT and Swin3D forwards are
    captured and replayed on two streams: logits bit-identical to the eager forward, and another
    collective still runs afterwards."""
    from vclip_amd.swin3d import Swin3d
    from vclip_amd.vivit import VivitConfig, VivitForVideoClassification
    from vclip_amd.weights import make_swin3d_weights, make_synthetic_clips, make_synthetic_video, make_vivit_weights
    t = torch.ones(4, device="cuda")
    rccl.all_reduce(t)  # the communicator and its watchdog are live
    torch.cuda.synchronize()
    vm = VivitForVideoClassification(VivitConfig(**CFG, id2label={0: "a", 1: "b"}))
    vm.load_state_dict(make_vivit_weights(CFG, seed=0))
    vm = vm.cuda().eval()
    pix = torch.from_numpy(make_synthetic_clips(2, 4, 32, seed=1)).cuda()
    swin_cfg = dict(patch_size=(2, 4, 4), embed_dim=32, depths=(2, 2), num_heads=(1, 2), window_size=(2, 3, 3),
                    mlp_ratio=4.0, layer_norm_eps=1e-5, num_classes=2)
    sm = Swin3d({k: v for k, v in swin_cfg.items() if k != "num_classes"}, num_classes=2)
    sm.load_state_dict(make_swin3d_weights(swin_cfg, seed=0))
    sm = sm.cuda().eval()
    video = torch.from_numpy(make_synthetic_video(2, 8, 48, seed=4)).cuda()
    for m, x in ((vm, pix), (sm, video)):
        m.concurrent_streams = 2
        want = m.forward_logits(x).clone()
        m.graph_replay = True
        for _ in range(3):
            assert torch.equal(m.forward_logits(x), want)
        assert m._graphs.captures == 1
        m.graph_replay = False
    rccl.all_reduce(t)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.ones(4))  # world 1: the sum is the identity
