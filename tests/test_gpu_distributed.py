"""RCCL (torch.distributed "nccl" on ROCm) path of the sharded feature cache on the GPU box:
a world_size-1 process group over the real HIP model. sharded_encode /
compute_image_features_sharded give the plain encode bit for bit,
the collective runs on the rank's HIP device whatever device the loader's
images are on (CPU batches here, like a DataLoader's), and the timed bench
step uses exactly this function."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_encode_rccl_world1():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import miclip
    from miclip.feature_cache import compute_image_features_sharded, sharded_encode
    from miclip.weights import synthetic_images
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda:0"))
    try:
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        _, m, _ = miclip.load("ViT-B/32", device="cuda")
        imgs = torch.from_numpy(synthetic_images(37, 224, seed=4))           # host batch
        ref = m.encode_image(imgs.cuda(), normalize=True)
        got = sharded_encode(lambda x: m.encode_image(x, normalize=True), imgs, dim=768)
        assert got.device.type == "cuda" and torch.equal(got, ref)
        got_dev = sharded_encode(lambda x: m.encode_image(x, normalize=True), imgs.cuda(), dim=768)
        assert torch.equal(got_dev, ref)
        loader = [(imgs[i:i + 10], torch.arange(i, min(i + 10, 37))) for i in range(0, 37, 10)]
        feats, labels = compute_image_features_sharded(m, loader, normalize=True)
        assert torch.equal(feats, ref) and torch.equal(labels.cpu(), torch.arange(37))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_cache_gloo_world2_one_gpu():
    """Two ranks (torch.distributed.run, gloo over 127.0.0.1) share the one GPU of the
    box, each running its own HIP model on cuda:0: the sharded encode and both
    sharded feature-cache loader forms equal the single-process encode bit for bit
    on every rank (tests/dist_gpu_worker.py). The ranks are started as child
    processes (no exec from this GPU-initialised process)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "tests", "dist_gpu_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "RANK_OK 0" in out and "RANK_OK 1" in out, out[-3000:]


@pytest.mark.timeout(300)
def test_bench_two_rank_rehearsal():
    """bench.py's N-rank logic on the box (the driver's 8-GPU run is not ours to start):
    torch.distributed.run with two ranks, gloo collectives, both ranks on the one GPU
    (--rehearse-gloo). Rank 0 prints one JSON line for the world of 2, marked as a
    rehearsal; the step's guard against the single-GPU encode ran on both ranks."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4", MICLIP_QUIET="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--rehearse-gloo", "--model", "ViT-B/32",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=root)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0 and "rehearsal" in d
    assert d["config"]["global_batch"] == 256 and d["config"]["images_per_gpu"] == 128
