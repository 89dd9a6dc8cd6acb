"""CPU, world_size 2 (gloo): the product's sharded feature-cache path
(miclip.feature_cache.compute_image_features_sharded -> sharded_encode ->
all_gather_into_tensor) reproduces the single-process compute_image_features
row for row (row order aihab_utils/feature_cache.py:144-162),
including batches smaller than the world (a rank with an empty shard).

The HIP model needs a GPU, so the encoder here is a deterministic stand-in with
the model surface the drivers use (parameters() for device inference,
config.vision_width, encode_image(x, normalize=...)); its rows depend on their
own image only, like the real encoder (checked bitwise on the GPU by
tests/test_gpu_parity.py::test_batch_invariance_and_shards and
tests/test_gpu_distributed.py).
"""
import os
import socket
from types import SimpleNamespace

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


class StubCLIP(torch.nn.Module):
    """Row-wise encoder: a fixed nonlinear map of each image + optional L2 norm."""

    def __init__(self, width=8):
        super().__init__()
        self.config = SimpleNamespace(vision_width=width)
        self.w = torch.nn.Parameter(torch.linspace(-1, 1, 3 * 4 * 4).view(-1, 1) *
                                    torch.arange(1, width + 1).view(1, -1), requires_grad=False)

    @torch.no_grad()
    def encode_image(self, x, normalize=False):
        y = torch.tanh(x.flatten(1) @ self.w)
        return torch.nn.functional.normalize(y, dim=-1) if normalize else y


def _batches(sizes):
    g = torch.Generator().manual_seed(0)
    out, label = [], 0
    for n in sizes:
        out.append((torch.randn(n, 3, 4, 4, generator=g), torch.arange(label, label + n)))
        label += n
    return out


def _worker(rank, world, port, sizes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from miclip.feature_cache import compute_image_features_sharded, sharded_encode
    model = StubCLIP()
    feats, labels = compute_image_features_sharded(model, _batches(sizes), normalize=True)
    one = sharded_encode(lambda x: model.encode_image(x), torch.randn(1, 3, 4, 4), dim=8)
    q.put((rank, feats.numpy(), labels.numpy(), str(feats.device), str(one.device), tuple(one.shape)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [[6, 7, 1], [1], [5, 2, 3]])
def test_sharded_feature_cache_matches_single_process(sizes):
    from miclip.feature_cache import compute_image_features
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    model = StubCLIP()
    ref_f, ref_l = compute_image_features(
        SimpleNamespace(parameters=model.parameters,
                        encode_image=lambda x: model.encode_image(x, normalize=True)),
        _batches(sizes))
    for r in range(world):
        feats, labels, fdev, onedev, oneshape = res[r]
        assert fdev == "cpu" and onedev == "cpu" and oneshape == (1, 8)
        assert feats.shape == tuple(ref_f.shape)
        assert (feats == ref_f.numpy()).all(), "gathered rows differ from the single-process cache"
        assert (labels == ref_l.numpy()).all()


class _LoggedDataset:
    """(image, label) items; records which indices this process read."""

    def __init__(self, n):
        g = torch.Generator().manual_seed(1)
        self.x = torch.randn(n, 3, 4, 4, generator=g)
        self.read = []

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        self.read.append(i)
        return self.x[i], i + 100


def _worker_per_rank(rank, world, port, n, bs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from miclip.feature_cache import ShardedBatchLoader, compute_image_features_sharded
    ds = _LoggedDataset(n)
    loader = ShardedBatchLoader(ds, bs)
    feats, labels = compute_image_features_sharded(StubCLIP(), loader, normalize=True, per_rank=True)
    q.put((rank, feats.numpy(), labels.numpy(), sorted(ds.read)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,bs", [(13, 6), (1, 4), (9, 3), (8, 8)])
def test_per_rank_loader_matches_single_process(n, bs):
    """Each rank reads and decodes only its contiguous slice of every global batch
    (ShardedBatchLoader); gather_shards restores the single-process row order of
    features and labels (aihab_utils/feature_cache.py:144-162)."""
    from miclip.feature_cache import compute_image_features, shard_range
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker_per_rank, args=(r, world, port, n, bs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ds = _LoggedDataset(n)
    batches = [(ds.x[b:b + bs], torch.arange(b, min(n, b + bs)) + 100) for b in range(0, n, bs)]
    model = StubCLIP()
    ref_f, ref_l = compute_image_features(
        SimpleNamespace(parameters=model.parameters,
                        encode_image=lambda x: model.encode_image(x, normalize=True)), batches)
    for r in range(world):
        feats, labels, read = res[r]
        want = []
        for b in range(0, n, bs):
            lo, hi = shard_range(min(bs, n - b), r, world)
            want += list(range(b + lo, b + hi))
        assert read == want, "a rank read images outside its own slice"
        assert (feats == ref_f.numpy()).all() and (labels == ref_l.numpy()).all()


def _worker_counts(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from miclip.feature_cache import gather_shards, shard_range
    n = 7
    counts = [b - a for a, b in (shard_range(n, r, world) for r in range(world))]
    lo, hi = shard_range(n, rank, world)
    local = torch.arange(lo * 3, hi * 3, dtype=torch.float32).view(-1, 3)
    got = gather_shards(local, counts=counts)            # known counts: no count exchange
    got2 = gather_shards(local)                          # exchanged counts
    err = None
    try:
        gather_shards(local, counts=[counts[0] + 1] + counts[1:] if rank == 0 else counts[::-1])
    except ValueError as e:
        err = str(e)
    q.put((rank, got.numpy(), got2.numpy(), err))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_shards_known_counts():
    """gather_shards(counts=...) (bench.py's step: the slices of a known batch) gives
    the exchanged-count result without its host sync; wrong counts are refused."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker_counts, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, a, b, err = q.get(timeout=120)
        res[r] = (a, b, err)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = torch.arange(21, dtype=torch.float32).view(7, 3).numpy()
    for r in range(world):
        a, b, err = res[r]
        assert (a == want).all() and (b == want).all()
        assert err is not None and "counts" in err
