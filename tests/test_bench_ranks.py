"""CPU: bench.py's rank logic at world 2 over gloo (the code the driver's 8-GPU
run executes: process-group setup, the sharded step through sharded_encode's
all-gather, the correctness guard against the single-GPU encode, the barriers
around the timed steps, the all_reduce(MAX) of the step time and the teardown).

bench.run takes the backend and the model loader as arguments (default: nccl =
RCCL and miclip.load); here gloo on the host and a row-wise stand-in encoder
with the model surface bench.py calls, since the HIP model needs a GPU.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class StubModel:
    """encode_image: 14x14 average pool of a 224px image = 3*16*16 = 768 features
    per image (ViT-B/32's width), tanh, optional L2 norm -- each row depends on its
    own image only, like the real encoder."""

    def __init__(self):
        g = torch.Generator().manual_seed(3)
        self.proj = torch.randn(768, 512, generator=g) / 28.0
        self.calls = 0

    def reserve(self, *a):
        pass

    def set_splits(self, s):
        pass

    def image_splits(self, n):
        return 1

    def numerics(self):
        return dict(resid16=True, lnfold=True, lnfold_text=True, mxfp8=False, cls_last=True, mx_out=False,
                    mx_gelu_tanh=False)

    def encode_text(self, toks):
        g = torch.Generator().manual_seed(int(toks.sum()) % 1000)
        xp = torch.randn(toks.shape[0], 512, generator=g)
        return xp.clone(), xp

    def encode_image(self, x, normalize=False):
        self.calls += 1
        y = torch.tanh(F.avg_pool2d(x, 14).flatten(1))
        return F.normalize(y, dim=-1) if normalize else y

    def zero_shot(self, feats, tw, scale=100.0, k=1, apply_proj=True):
        f = feats @ self.proj if apply_proj else feats
        logits = scale * F.normalize(f, dim=-1) @ tw
        return logits, logits.topk(k, dim=1).indices


def _stub_loader(name, dev, dtype, options=None):
    return StubModel()


ARGV = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "4", "--model", "ViT-B/32",
        "--classes", "5", "--no-profile", "--no-cpu-baseline"]


def _rank(rank, world, port, q, extra):
    import torch.distributed as dist
    import bench
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    line = bench.run(bench.parse(ARGV + extra), backend="gloo", load_model=_stub_loader)
    q.put((rank, line, dist.is_initialized()))


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_rank_logic_world2_gloo(scaling):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    extra = [] if scaling == "strong" else ["--scaling", "weak"]     # strong is the default
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, extra)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, line, still = q.get(timeout=180)
        res[r] = (line, still)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    line0, still0 = res[0]
    line1, still1 = res[1]
    assert line1 is None and not still0 and not still1     # rank 0 reports; groups torn down
    assert line0["n_gpus"] == 2 and line0["steps"] == 2 and line0["warmup"] == 1
    assert line0["scaling"] == scaling and line0["value"] > 0
    if scaling == "weak":     # --batch images per GPU
        assert line0["config"]["global_batch"] == 8 and line0["config"]["images_per_gpu"] == 4
        assert "weak_scaling" not in line0
    else:                     # the global --batch split over the ranks
        assert line0["config"]["global_batch"] == 4 and line0["config"]["images_per_gpu"] == 2
        w = line0["weak_scaling"]             # plus the weak figure of the same run
        assert w["global_batch"] == 8 and w["images_per_gpu"] == 4 and w["value"] > 0
    n = line0["config"]["global_batch"]
    assert line0["value"] == pytest.approx(n * 2 / (line0["ms_per_step"] * 2 / 1e3), rel=1e-2)
    assert line0["clock_ghz"] is None and line0["roofline"] is None     # no HIP device here


def test_bench_rank_logic_world1_host(monkeypatch):
    import bench
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    argv = [a if a != "2" or i != 1 else "1" for i, a in enumerate(ARGV)]
    line = bench.run(bench.parse(argv), backend="gloo", load_model=_stub_loader)
    assert line["n_gpus"] == 1 and line["config"]["global_batch"] == 4
    assert line["gflop_per_image_executed"] < line["gflop_per_image"]
