#!/usr/bin/env python
"""Benchmark: images/sec of the CLIP feature-cache encode on MI355X.

One step = the hot path of the reference's feature-cache loop
(aihab_utils/feature_cache.py:114-142 / methods/utils.py:142-173) over one
device-resident global batch, sharded by image as the product's per-rank
driver does (ShardedBatchLoader + gather_shards):
    each rank holds and encodes only its contiguous slice (encode_image, all
    HIP kernels, L2-normalise fused into ln_post)
    -> RCCL all-gather of the normalised embeddings back into the global row
       order (miclip.feature_cache.gather_shards; N > 1;
       aihab_utils/feature_cache.py:144-162)
    -> zero-shot logits of the gathered rows (x @ visual.proj -> normalise
       -> 100 * f @ text_weights -> top-1; methods/ProLIP.py:288-293).
--scaling strong (default): global batch 256 split 256/N per GPU
(256/128/64/32 images per rank at N = 1/2/4/8); at N > 1 the line also carries
the weak-scaling figure (256 images per GPU) timed in the same run.
--scaling weak: 256 images per GPU, global batch 256 N.
`value` = global images per step * K / max-over-ranks wall time of the K steps.

`python bench.py --gpus N` starts the N ranks itself (one process per GPU,
spawned before anything touches the GPU); under torchrun (WORLD_SIZE set) it
is one of the ranks. n_gpus is the world size RCCL actually formed.

Also reported (rank 0): the dominant kernel's roofline (MLP c_fc GEMM:
algorithmic FLOPs / its average launch time from HIP events of one profiled
step, which runs the batch unsplit on one stream; traffic from the committed
PMC profile of that same kernel and launch shape, else null), the whole-path
MFMA fraction, and the reference CPU encode (the repo's fp32 torch-CPU
restatement of clip/model.py, oracle/clip_oracle.py, bit-exact with the
reference on the same machine) timed on this host on a bounded sample.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong]
                    [--model ViT-L/14] [--batch 256] [--ab-splits] [--ab-fold]
"""
import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "aihab-clip_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "images/sec encoded (ViT-L/14 bs=256) at 1/2/4/8 GPUs; % bf16 MFMA roofline"
PEAK_TFLOPS = 256 * 2.4e9 * 4096 / 1e12   # dense bf16/fp16 MFMA, MI355X_MICROARCH.md
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "traffic_gemm_fc.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"])
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="one-GPU rehearsal of the N-rank logic: gloo collectives, every rank on "
                         "cuda:(LOCAL_RANK mod devices); the line is marked, its value is not a "
                         "multi-GPU result")
    ap.add_argument("--no-weak", action="store_true",
                    help="N > 1 strong runs: skip the secondary weak-scaling measurement")
    ap.add_argument("--model", default="ViT-L/14")
    ap.add_argument("--batch", type=int, default=256,
                    help="images per GPU (weak) or global images (strong) per step")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "mxfp8"])
    ap.add_argument("--classes", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--splits", type=int, default=2, help="encode_image batch split over streams")
    ap.add_argument("--ab-splits", action="store_true", help="also time splits=1 vs 2 (diagnostic)")
    ap.add_argument("--ab-gemm", default="",
                    help="diagnostic: also time these GEMM variants 'ln:res[:mx],...' (e.g. "
                         "'0:0,508:0' or '0:0:1,0:0:2' for the MX-fp8 kernels) interleaved in "
                         "this process (bit-identical kernels)")
    ap.add_argument("--ab-fold", action="store_true",
                    help="also time a second model with options ln_fold=False in this process (diagnostic)")
    ap.add_argument("--ab-options", default="",
                    help="diagnostic: also time a second model with these options "
                         "('name=0|1,...', e.g. 'resid_f32=1') interleaved in this process")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher --

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_entry(rank, world, port, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(parse(argv))


def spawn(args, argv):
    """One process per GPU, started before this process touches the GPU."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, args.gpus, port, argv)) for r in range(args.gpus)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    codes = [p.exitcode for p in procs]
    if any(codes):
        log(f"[bench] rank exit codes {codes}")
    return max((abs(c) for c in codes if c), default=0)


# ------------------------------------------------------------- CPU baseline --

def cpu_baseline(model, cfg, budget_s=12.0, max_images=64):
    """Time the fp32 torch-CPU oracle (reference arithmetic) on a bounded sample."""
    import torch
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


# ---------------------------------------------------------------- roofline --

def _lib_label():
    from miclip import _lib
    here = os.path.relpath(_lib.LIB_PATH, ROOT) if _lib.LIB_PATH.startswith(ROOT) else _lib.LIB_PATH
    return here if "MICLIP_LIB" in os.environ else f"{here} (in-tree build)"


def fc_epilogue(numerics):
    """The c_fc GEMM's epilogue functor as it appears in the kernel symbol."""
    if numerics["mxfp8"]:
        return "EpiMX"
    return "EpiStoreLN" if numerics["lnfold"] else "EpiStore"


def attach_traffic(model_name, dtype, epi, M):
    """HBM-side bytes per launch from the committed PMC profile, only when it was
    taken on the same kernel (epilogue), model, dtype and launch shape."""
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, "no profile"
    want = {"model": model_name, "dtype": dtype, "epilogue": epi, "M": M}
    got = {k: t.get(k) for k in want}
    if got != want:
        return None, f"profile is for {got}, run is {want}"
    return t.get("hbm_bytes_per_launch"), t.get("source")


# --------------------------------------------------------------------- rank --

def _load_miclip(name, dev, dtype, options=None):
    import warnings
    import miclip
    # OpenAI surface for every model (pre-projection encode, projection in the head);
    # seeded random weights are the bench's stated synthetic data ("data" field)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", miclip.SeededWeightsWarning)
        _, model, _ = miclip.load(name, device=dev, compute_dtype=dtype, surface="openai",
                                  options=options)
    return model


class ClockProbe:
    """Core clock the chip held over a timed region (miclip_clock_probe): one-wave
    workgroups on the timed stream read s_memtime (shader-clock counter) and
    s_memrealtime (100 MHz) before and after; per XCD (HW_REG_XCC_ID)
    delta(memtime) / delta(realtime) x 100 MHz, median over the XCDs."""

    NWG = 512         # 64 per XCD under round-robin dispatch (medians over many CUs)
    MIN_WINDOW_S = 0.1
    GHZ_RANGE = (1.0, 2.4)   # MI355X core clock floor under load .. nameplate maximum

    def __init__(self, dev):
        import torch
        from miclip import _lib
        self.lib = _lib.load_library()
        self.torch = torch
        self.dev = dev
        self.buf = torch.zeros(2, self.NWG, 4, dtype=torch.int64, device=dev)

    def mark(self, i):
        from miclip import _lib
        _lib.check(self.lib.miclip_clock_probe(self.buf[i].data_ptr(), self.NWG,
                                               _lib.stream_handle(self.dev)), "miclip_clock_probe")

    def ghz(self):
        import numpy as np
        b = self.buf.cpu().numpy()
        per_xcd = {}
        for x in np.unique(b[0, :, 0]):
            a0, a1 = b[0][b[0, :, 0] == x], b[1][b[1, :, 0] == x]
            if len(a0) == 0 or len(a1) == 0:
                continue
            dt = float(np.median(a1[:, 1]) - np.median(a0[:, 1]))
            dr = float(np.median(a1[:, 2]) - np.median(a0[:, 2]))
            if dr > 0:
                per_xcd[int(x)] = dt / dr * 0.1        # GHz (realtime ticks at 100 MHz)
        # a physically impossible reading (CU counter offsets across the window)
        # is reported as rejected, never folded into the median
        lo, hi = self.GHZ_RANGE
        ok = {k: v for k, v in per_xcd.items() if lo <= v <= hi}
        rej = {k: round(v, 4) for k, v in sorted(per_xcd.items()) if k not in ok}
        if not ok:
            return None, {}, rej
        vals = sorted(ok.values())
        return (round(float(np.median(vals)), 4), {k: round(v, 4) for k, v in sorted(ok.items())},
                rej)


def run(args, backend="nccl", load_model=None):
    """One rank of the bench. backend "nccl" (RCCL, the product) on the rank's HIP
    device; "gloo" runs the same rank logic on the host (tests/test_bench_ranks.py
    drives it at world 2 with a stub model). Returns rank 0's JSON line (dict)."""
    import torch
    import torch.distributed as dist

    rehearse = bool(getattr(args, "rehearse_gloo", False))
    on_gpu = backend == "nccl" or rehearse
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        elif on_gpu:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()            # the group the backend actually formed
        rank = dist.get_rank()
    if args.gpus != world and rank == 0:
        log(f"[bench] --gpus {args.gpus} but the process group has {world} ranks; reporting {world}")
    if on_gpu:
        if rehearse:
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
    else:
        dev = torch.device("cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    from miclip.configs import MODEL_CONFIGS, algorithmic_gflop_per_image, executed_gflop_per_image
    from miclip.feature_cache import gather_shards, shard_range
    from miclip.weights import CLIP_MEAN, CLIP_STD
    cfg = MODEL_CONFIGS[args.model]
    R, W = cfg.image_resolution, cfg.vision_width
    n_global = args.batch * world if args.scaling == "weak" else args.batch
    lo, hi = shard_range(n_global, rank, world)
    t_load = time.perf_counter()
    load_model = load_model or _load_miclip
    model = load_model(args.model, dev, args.dtype)
    peak = PEAK_TFLOPS * (2 if args.dtype == "mxfp8" else 1)   # MX-fp8 runs at 2x the f16 rate
    model.reserve(max(hi - lo, 1), args.classes)
    model.set_splits(args.splits)
    log(f"[rank {rank}] model loaded in {time.perf_counter() - t_load:.1f}s; "
        f"{hi - lo} of {n_global} images per step on this rank")

    # synthetic CLIP-normalised images, device-resident before timing. Each rank
    # makes only its own slice [lo, hi) of the global batch, as a per-rank loader
    # does (feature_cache.ShardedBatchLoader): image i comes from the generator of
    # its 256-image chunk, so it is the same image on whichever rank makes it
    mean = torch.tensor(CLIP_MEAN, device=dev).view(1, 3, 1, 1)
    std = torch.tensor(CLIP_STD, device=dev).view(1, 3, 1, 1)

    def make_images(a, b, n_all=n_global):
        out = torch.empty(max(b - a, 0), 3, R, R, device=dev)
        for c in range(a // 256, (b + 255) // 256):
            g = torch.Generator(device=dev).manual_seed(1234 + c)
            u = torch.rand(min(256, n_all - 256 * c), 3, R, R, device=dev, generator=g)
            s0, s1 = max(a, 256 * c), min(b, 256 * c + u.shape[0])
            out[s0 - a:s1 - a] = (u[s0 - 256 * c:s1 - 256 * c] - mean) / std
        return out

    imgs = make_images(lo, hi)
    counts = [b - a for a, b in (shard_range(n_global, r, world) for r in range(world))]

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

    def make_step(m, imgs=imgs, counts=counts):
        has = imgs.shape[0] > 0

        def step():
            # this rank's slice, then the RCCL all-gather of the L2-normalised rows
            # back into the global order (gather_shards), then the zero-shot head
            local = m.encode_image(imgs, normalize=True) if has else None
            feats = gather_shards(local, width=W, counts=counts)   # [n_global, W]
            return m.zero_shot(feats, tw, 100.0, k=1, apply_proj=True)
        return step

    step = make_step(model)

    def timed(fn, steps, clock=None):
        sync()
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        if clock is not None:
            clock.mark(0)
        for _ in range(steps):
            fn()
        if clock is not None:
            clock.mark(1)
        sync()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        dt_t = torch.tensor([dt], device="cpu" if rehearse else dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        return float(dt_t.item())

    def clock_window(fn, per_step_s):
        """A clock reading over >= ClockProbe.MIN_WINDOW_S of back-to-back steps
        (untimed): the probe's per-XCD deltas come from different CUs before and
        after, so a short window magnifies their counter offsets."""
        n = max(1, int(ClockProbe.MIN_WINDOW_S / max(per_step_s, 1e-6)) + 1)
        c = ClockProbe(dev)
        timed(fn, n, c)
        return c, n

    # correctness guard on the timed path: the first 4 rows of every rank's slice,
    # gathered, are the single-GPU encode of those images in global order
    if world > 1:
        k = min(4, hi - lo)
        firsts = [shard_range(n_global, r, world) for r in range(world)]
        chk = gather_shards(model.encode_image(imgs[:k], normalize=True) if k else None, width=W,
                            counts=[min(4, b - a) for a, b in firsts])
        ref_imgs = torch.cat([make_images(a, min(a + 4, b)) for a, b in firsts])
        ref = model.encode_image(ref_imgs, normalize=True)
        assert torch.equal(chk.to(ref.device), ref), "gathered rows differ from the single-GPU encode"
        del ref_imgs

    for _ in range(args.warmup):
        step()
    clock = ClockProbe(dev) if on_gpu else None
    dt = timed(step, args.steps, clock)
    value = n_global * args.steps / dt
    clock_steps = args.steps
    if clock is not None and dt < ClockProbe.MIN_WINDOW_S:
        # the timed region is too short for the probe: read the clock over a
        # longer run of the same step right after it
        clock, clock_steps = clock_window(step, dt / args.steps)
    clock_ghz, clock_xcd, clock_rej = clock.ghz() if clock is not None else (None, {}, {})

    weak = None
    if args.scaling == "strong" and world > 1 and not args.no_weak:
        # the weak-scaling figure of the same run: --batch (256) images per GPU
        n_w = args.batch * world
        wlo, whi = shard_range(n_w, rank, world)
        model.reserve(whi - wlo, args.classes)
        wstep = make_step(model, make_images(wlo, whi, n_w),
                          [b - a for a, b in (shard_range(n_w, r, world) for r in range(world))])
        for _ in range(max(args.warmup, 1)):
            wstep()
        wsteps = max(3, args.steps * (hi - lo) // 256)
        wdt = timed(wstep, wsteps)
        weak = {"value": round(n_w * wsteps / wdt, 2), "images_per_gpu": whi - wlo,
                "global_batch": n_w, "steps": wsteps, "ms_per_step": round(wdt / wsteps * 1e3, 3),
                "path_mfma_frac": None}
        del wstep
    gf = algorithmic_gflop_per_image(cfg)
    cls_last = model.numerics()["cls_last"]
    gf_exec = executed_gflop_per_image(cfg, cls_last=cls_last)

    ab = None
    if args.ab_splits:
        ab = {}
        for sp in (1, 2, 3, 1, 2, 3):
            model.set_splits(sp)
            eff = model.image_splits(max(hi - lo, 1))   # the part count actually run
            step()
            ab.setdefault(f"splits{sp}" + (f"_ran{eff}" if eff != sp else ""), []).append(
                round(n_global * args.steps / timed(step, args.steps), 1))
        model.set_splits(args.splits)
    abg = None
    if args.ab_gemm:
        abg = {}
        pairs = [tuple(int(x) for x in p.split(":")) for p in args.ab_gemm.split(",")]
        for _ in range(3):
            for pv in pairs:
                for which, v in enumerate(pv):      # ln:res[:mx]
                    model.set_gemm_variant(which, v)
                step()
                abg.setdefault(":".join(map(str, pv)), []).append(
                    round(n_global * args.steps / timed(step, args.steps), 1))
        for which in range(3):
            model.set_gemm_variant(which, 0)
        abg = {k: dict(runs=v, median=statistics.median(v)) for k, v in abg.items()}
    abf = None
    if args.ab_fold or args.ab_options:
        alt = ({"ln_fold": False} if args.ab_fold else
               {k: bool(int(v)) for k, v in (p.split("=") for p in args.ab_options.split(","))})
        m0 = load_model(args.model, dev, args.dtype, options=alt)
        m0.reserve(max(hi - lo, 1), args.classes)
        m0.set_splits(args.splits)
        step0 = make_step(m0)
        step0()
        # "fold" = this run's model, "nofold" = the alternative options (the names
        # are the --ab-fold ones; `alt_options` says what the alternative was)
        abf = {"fold": [], "nofold": [], "fold_flags": model.numerics(), "nofold_flags": m0.numerics(),
               "alt_options": alt}
        for _ in range(3):
            abf["fold"].append(round(n_global * args.steps / timed(step, args.steps), 1))
            abf["nofold"].append(round(n_global * args.steps / timed(step0, args.steps), 1))
        abf["fold_median"] = statistics.median(abf["fold"])
        abf["nofold_median"] = statistics.median(abf["nofold"])
        del m0, step0
        if on_gpu:
            torch.cuda.empty_cache()

    roofline, kernels = None, None
    prof = None
    if not args.no_profile:
        # every rank runs the profiled step (it contains the all-gather); profiling
        # runs each rank's batch unsplit on one stream, so a GEMM launch has M = b*N
        model.set_profiling(True)
        step()
        sync()
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
            M = (hi - lo) * cfg.n_tokens
            epi = fc_epilogue(model.numerics())
            traffic, tsrc = attach_traffic(args.model, args.dtype, epi, M)
            nm = model.numerics()
            act_name = ("QuickGELU" if cfg.act != "erf" else
                        "GELU, tanh form" if nm.get("mxfp8") and nm.get("mx_gelu_tanh") else "exact GELU")
            roofline = {"bound": "mfma", "achieved": round(achieved, 1), "peak": round(peak, 1),
                        "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                        "kernel": f"gemm_fc: MLP c_fc GEMM, {epi} epilogue + {act_name}"
                                  + (" (ln_2 folded in)" if epi == "EpiStoreLN" else ""),
                        "launch": {"M": M, "N": 4 * W, "K": W, "splits": 1,
                                   "timing": "HIP events on the launch stream, profiled step"},
                        "algorithmic_flops_per_launch": flops_launch,
                        "avg_launch_ms": round(per_launch_s * 1e3, 4),
                        "traffic_source": tsrc}
    if roofline is not None:
        # the clock held over the timed steps (not the profiled one): the peak
        # scales with it (2.4 GHz nameplate), so frac_at_clock separates the
        # kernel's schedule from the chip's DVFS state on this box
        roofline["clock_ghz"] = clock_ghz
        roofline["clock_ghz_per_xcd"] = clock_xcd
        roofline["clock_source"] = (
            "miclip_clock_probe: s_memtime / s_memrealtime per XCD, before and after "
            + ("the timed steps" if clock_steps == args.steps else
               f"{clock_steps} back-to-back steps right after the timed ones (timed region "
               f"< {ClockProbe.MIN_WINDOW_S} s)")
            + f" on the bench stream; XCD readings outside {ClockProbe.GHZ_RANGE} GHz rejected")
        roofline["clock_rejected_per_xcd"] = clock_rej
        roofline["frac_at_clock"] = (round(roofline["frac"] * 2.4 / clock_ghz, 4)
                                     if clock_ghz else None)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(model, cfg, budget_s=args.cpu_seconds)

    if rank == 0:
        per_gpu = f"{args.batch}/GPU" if args.scaling == "weak" else f"{n_global}/{world} per GPU"
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (224px CLIP-normalised uniform noise; seeded random-init weights)",
            "config": {"workload": f"{args.model} feature-cache encode: encode_image bs={per_gpu} "
                                   f"@{R}px + L2-normalise + RCCL all-gather (gather_shards) + "
                                   f"zero-shot logits ({args.classes} classes)",
                       "global_batch": n_global, "images_per_gpu": hi - lo,
                       "tokens_per_image": cfg.n_tokens,
                       "parallelism": f"dp{world} (image-batch sharding, {args.scaling} scaling)",
                       "splits": model.image_splits(max(hi - lo, 1)),
                       "splits_requested": args.splits, "numerics": model.numerics(),
                       "weights": "seeded random init, CLIP shapes",
                       # the library this run loaded (MICLIP_LIB overrides the in-tree
                       # build for A/B against another revision's binary)
                       "library": _lib_label()},
            "gflop_per_image": round(gf, 3),
            "path_mfma_frac": round(value * gf * 1e9 / (world * peak * 1e12), 4),
            # FLOPs the kernels execute (the last vision block runs on the CLS rows
            # only, clip/model.py:226-229): the algorithmic figure counts them all
            "gflop_per_image_executed": round(gf_exec, 3),
            "path_mfma_frac_executed": round(value * gf_exec * 1e9 / (world * peak * 1e12), 4),
            "clock_ghz": clock_ghz,
            "roofline": roofline, "cpu_baseline": cpu, "kernels": kernels,
        }
        if rehearse:
            line["rehearsal"] = (f"{world} ranks over gloo on {torch.cuda.device_count()} GPU(s): "
                                 "the multi-rank logic on hardware, not a scaling result")
        if ab:
            line["splits_ab_img_s"] = ab
        if abf:
            line["fold_ab_img_s"] = abf
        if abg:
            line["gemm_ab_img_s"] = abg
        if weak:
            weak["path_mfma_frac"] = round(weak["value"] * gf * 1e9 / (world * peak * 1e12), 4)
            line["weak_scaling"] = weak
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return line if rank == 0 else None


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn(args, argv))
    run(args)


if __name__ == "__main__":
    main()
