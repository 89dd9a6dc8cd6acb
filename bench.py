#!/usr/bin/env python
"""Benchmark: images/sec of the CLIP feature-cache encode on MI355X.

One step = the hot path of the reference's feature-cache loop
(aihab_utils/feature_cache.py:114-142 / methods/utils.py:142-173) on one
device-resident batch per GPU:
    encode_image (ViT, all HIP kernels) -> L2-normalise (fused into ln_post)
    -> RCCL all-gather of the normalised embeddings over the ranks (N > 1)
    -> zero-shot logits of the gathered rows (x @ visual.proj -> normalise
       -> 100 * f @ text_weights -> top-1; methods/ProLIP.py:288-293).
Per-GPU batch is fixed (weak scaling); `value` = all ranks' images / max-over-
ranks wall time of the K timed steps.

Also reported (rank 0): the dominant kernel's roofline (MLP c_fc GEMM,
algorithmic FLOPs / its average launch time from HIP events of one profiled
step), the whole-path MFMA fraction, and the reference CPU encode (the
repo's fp32 torch-CPU restatement of clip/model.py, oracle/clip_oracle.py,
bit-exact with the reference) timed on this host on a bounded sample.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model ViT-L/14] [--batch 256]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "aihab-clip_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec encoded (ViT-L/14 bs=256) at 1/2/4/8 GPUs; % bf16 MFMA roofline"
PEAK_TFLOPS = 256 * 2.4e9 * 4096 / 1e12   # dense bf16/fp16 MFMA, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(model, cfg, budget_s=12.0, max_images=64):
    """Time the fp32 torch-CPU oracle (reference arithmetic) on a bounded sample."""
    from oracle import clip_oracle
    from miclip.weights import synthetic_images
    cores = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(cores, int(omp)) if omp and omp.isdigit() else cores
    torch.set_num_threads(threads)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    chunk = 4
    warm = torch.from_numpy(synthetic_images(1, cfg.image_resolution, seed=99))
    clip_oracle.encode_image(sd, cfg, warm)
    done, t0 = 0, time.perf_counter()
    while done < max_images and (time.perf_counter() - t0) < budget_s:
        x = torch.from_numpy(synthetic_images(chunk, cfg.image_resolution, seed=100, offset=done))
        clip_oracle.encode_image(sd, cfg, x)
        done += chunk
    dt = time.perf_counter() - t0
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(done / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{done} images of {cfg.image_resolution}px encode_image, fp32 torch-CPU "
                      f"restatement of clip/model.py (oracle/clip_oracle.py), {dt:.1f}s, "
                      f"{threads} threads, {cpu_model}; baseline, not target"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="ViT-L/14")
    ap.add_argument("--batch", type=int, default=256, help="images per GPU per step")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "mxfp8"])
    ap.add_argument("--classes", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--splits", type=int, default=2, help="encode_image batch split over streams")
    ap.add_argument("--ab-splits", action="store_true", help="also time splits=1 vs 2 (diagnostic)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    import miclip
    from miclip.configs import MODEL_CONFIGS, algorithmic_gflop_per_image
    from miclip.weights import CLIP_MEAN, CLIP_STD
    cfg = MODEL_CONFIGS[args.model]
    B, R = args.batch, cfg.image_resolution
    t_load = time.perf_counter()
    _, model, _ = miclip.load(args.model, device=dev, compute_dtype=args.dtype)
    # dense MFMA peak of the GEMM operand type: MX-fp8 runs at twice the f16 rate
    peak = PEAK_TFLOPS * (2 if args.dtype == "mxfp8" else 1)
    model.reserve(B, args.classes)
    model.set_splits(args.splits)
    log(f"[rank {rank}] model loaded in {time.perf_counter() - t_load:.1f}s")

    # synthetic CLIP-normalised images, device-resident before timing
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    u = torch.rand(B, 3, R, R, device=dev, generator=g)
    mean = torch.tensor(CLIP_MEAN, device=dev).view(1, 3, 1, 1)
    std = torch.tensor(CLIP_STD, device=dev).view(1, 3, 1, 1)
    imgs = ((u - mean) / std).contiguous()
    del u

    # text head once (clip_classifier flow): synthetic prompt tokens -> encode_text
    gt = torch.Generator().manual_seed(7)
    L = cfg.context_length
    toks = torch.zeros(args.classes, L, dtype=torch.long)
    for c in range(args.classes):
        n = 8 + c % 40
        toks[c, 0] = 49406
        toks[c, 1:n - 1] = torch.randint(1, 49000, (n - 2,), generator=gt)
        toks[c, n - 1] = 49407
    _, temb = model.encode_text(toks.to(dev))
    tw = torch.nn.functional.normalize(temb, dim=-1).t().contiguous()      # [E, C]

    feats = torch.empty(B, cfg.vision_width, device=dev)
    gathered = torch.empty(world * B, cfg.vision_width, device=dev) if world > 1 else feats

    def step():
        model.encode_image(imgs, normalize=True, out=feats)
        if world > 1:
            dist.all_gather_into_tensor(gathered, feats)
        return model.zero_shot(gathered, tw, 100.0, k=1, apply_proj=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    value = world * B * args.steps / dt
    gf = algorithmic_gflop_per_image(cfg)

    ab = None
    if args.ab_splits:
        ab = {}
        for sp in (1, 2, 3, 4, 2, 3, 4):
            model.set_splits(sp)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            ab.setdefault(f"splits{sp}", []).append(round(world * B * args.steps / (time.perf_counter() - t1), 1))
        model.set_splits(args.splits)

    roofline, kernels = None, None
    prof = None
    if not args.no_profile:
        # every rank runs the profiled step: it contains the all-gather
        model.set_profiling(True)
        step()
        torch.cuda.synchronize()
        prof = model.profile_read(reset=True)
        model.set_profiling(False)
    if rank == 0 and prof is not None:
        kernels = {k: dict(launches=v["launches"], ms=round(v["ms"], 4),
                           tflops=round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1) if v["flops"] else None,
                           gbs=round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1))
                   for k, v in prof.items()}
        fc = prof.get("gemm_fc")
        if fc:
            per_launch_s = fc["ms"] * 1e-3 / fc["launches"]
            flops_launch = fc["flops"] / fc["launches"]
            achieved = flops_launch / per_launch_s / 1e12
            traffic = None
            tpath = os.path.join(ROOT, "profiles", "traffic_gemm_fc.json")
            if os.path.isfile(tpath):
                try:
                    with open(tpath) as f:
                        t = json.load(f)
                    if t.get("model") == args.model and t.get("batch") == B:
                        traffic = t.get("hbm_bytes_per_launch")
                except (OSError, ValueError):
                    traffic = None
            act_name = "exact-GELU" if cfg.act == "erf" else "QuickGELU"
            roofline = {"bound": "mfma", "kernel": f"gemm_fc (MLP c_fc + {act_name} epilogue)",
                        "achieved": round(achieved, 1), "peak": round(peak, 1),
                        "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                        "traffic": traffic,
                        "algorithmic_flops_per_launch": flops_launch,
                        "avg_launch_ms": round(per_launch_s * 1e3, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(model, cfg, budget_s=args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": f"{args.model} feature-cache encode: encode_image bs={B}/GPU "
                                   f"@{R}px + L2-normalise + RCCL all-gather + zero-shot "
                                   f"logits ({args.classes} classes)",
                       "global_batch": world * B, "tokens_per_image": cfg.n_tokens,
                       "parallelism": f"dp{world} (image-batch sharding)",
                       "weights": "seeded random init, CLIP shapes"},
            "gflop_per_image": round(gf, 3),
            "path_mfma_frac": round(value * gf * 1e9 / (world * peak * 1e12), 4),
            "roofline": roofline, "cpu_baseline": cpu, "kernels": kernels,
        }
        if ab:
            line["splits_ab_img_s"] = ab
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
