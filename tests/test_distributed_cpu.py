"""Multi-process (gloo, world size 2) test of the data-parallel extraction sharding: every frame is
processed by exactly one rank and the gathered feature bank equals the single-process one, in
order.  The per-frame 'extractor' here is a deterministic CPU stand-in (the real extractor needs
the GPU); what is under test is the shard/gather plumbing bench.py and the LFB writer use."""
import os
import socket

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


def _fake_features(idx):
    g = torch.Generator().manual_seed(0)
    w = torch.randn(1, 16, generator=g)
    return torch.sin(idx.float()[:, None] * w)


def _worker(rank, world, port, n, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deep-learning-for-surgical-video-analysis_amd"))
    from svk.shard import shard_range, gather_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard_range(n, rank, world)
    local = _fake_features(torch.arange(a, b))
    full = gather_rows(local, n)
    t = torch.tensor([float(b - a)])
    dist.all_reduce(t)
    out[rank] = (full.clone(), int(t.item()))
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [10, 7, 1])
def test_shard_gather_world2(n):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    ref = _fake_features(torch.arange(n))
    for r in range(world):
        full, total = out[r]
        assert total == n
        torch.testing.assert_close(full, ref)


def test_shard_range_properties():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deep-learning-for-surgical-video-analysis_amd"))
    from svk.shard import shard_range
    for n in (0, 1, 5, 1000, 98234):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _ddp_worker(rank, world, port, out, grad_comm="f32"):
    """The train step's data-parallel exchange (svk.train.EVPTrainStep.allreduce_grads over its two
    gradient buckets / sync_buffers) on CPU tensors: gradient averaging over ranks, BN buffers from
    rank 0."""
    import sys
    import types
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deep-learning-for-surgical-video-analysis_amd"))
    from svk.train import EVPTrainStep
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    grad = torch.randn(1000, generator=g)
    local = grad.clone()
    bns = [torch.nn.BatchNorm2d(8) for _ in range(5)]
    for i, bn in enumerate(bns):
        bn.running_mean.fill_(rank * 10.0 + i)
        bn.running_var.fill_(rank + 1.0)
    model = types.SimpleNamespace(head=types.SimpleNamespace(linear_fuse=types.SimpleNamespace(bn=bns[0])),
                                  flow_encoder=types.SimpleNamespace(**{f"bn{i}": bns[i] for i in range(1, 5)}))
    tr = EVPTrainStep.__new__(EVPTrainStep)     # the exchange methods only, no GPU state
    tr.group, tr.world, tr.grad, tr.model, tr.head_end = dist.group.WORLD, world, grad, model, 400
    tr.grad_comm, tr._comm = grad_comm, {}
    assert [b.numel() for b in tr._grad_buckets()] == [400, 600]      # head bucket, then the rest
    tr.allreduce_grads()
    tr.sync_buffers()
    out[rank] = (local, grad.clone(), [bn.running_mean.clone() for bn in bns], [bn.running_var.clone() for bn in bns])
    dist.destroy_process_group()


@pytest.mark.parametrize("grad_comm", ["f32", "bf16"])
def test_train_ddp_exchange_world2(grad_comm):
    """f32: the exact average; bf16 (SURVEY.md §5's compressed all-reduce): each rank's bucket rounded to bf16,
    summed, widened back — within bf16's relative rounding of the exact average, identical on every rank."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_ddp_worker, args=(world, _free_port(), out, grad_comm), nprocs=world, join=True)
    avg = (out[0][0] + out[1][0]) / 2
    tol = dict(rtol=0, atol=0) if grad_comm == "f32" else dict(rtol=2 ** -7, atol=2 ** -7 * float(avg.abs().max()))
    torch.testing.assert_close(out[0][1], out[1][1], rtol=0, atol=0)
    for r in range(world):
        if grad_comm == "f32":
            torch.testing.assert_close(out[r][1], avg)
        else:
            torch.testing.assert_close(out[r][1], avg, **tol)
            assert not torch.equal(out[r][1], avg)          # the bf16 path really ran
        for i in range(5):
            torch.testing.assert_close(out[r][2][i], torch.full((8,), float(i)))      # rank 0's buffers
            torch.testing.assert_close(out[r][3][i], torch.ones(8))
