"""CPU, world_size 2 (gloo): image-batch sharding + all-gather reproduces the
single-process result row for row (the multi-GPU feature cache path)."""
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


def _encode(x):
    # stand-in encoder (the C ABI needs a GPU): a fixed nonlinear row map + L2 norm
    w = torch.linspace(-1, 1, x[0].numel()).view(-1, 1) * torch.arange(1, 9).view(1, -1)
    return torch.nn.functional.normalize(torch.tanh(x.flatten(1) @ w), dim=-1)


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from miclip.feature_cache import sharded_encode
    g = torch.Generator().manual_seed(0)
    images = torch.randn(n, 3, 4, 4, generator=g)
    out = sharded_encode(_encode, images, dim=8)
    q.put((rank, out.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [6, 7, 1])
def test_sharded_encode_matches_single_process(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = torch.Generator().manual_seed(0)
    ref = _encode(torch.randn(n, 3, 4, 4, generator=g)).numpy()
    for r in range(world):
        assert res[r].shape == ref.shape
        assert (res[r] == ref).all()
