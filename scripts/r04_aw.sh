#!/bin/bash
# r04: one-head-per-workgroup attention balance -- head dim 64 (N = 577, C4) at up to
# 16 waves, head dim 80 (N = 257, C5) with the ragged last chunk split over the waves:
# attention tests, C4 / C5 parity, the probes, C4 / C5 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04aw
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 2 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 500 $PYT tests/test_gpu_kernels.py -k "attention"
step parity 700 $PYT tests/test_gpu_parity.py tests/test_gpu_largebatch.py tests/test_gpu_openclip.py -k "336 or c4 or vith14 or H-14 or openclip"
step probe 300 python scripts/probe/attn_waves.py 128 577 1,10,12,16
step ops80 300 python scripts/bench_ops.py --ops attention --batch 256 --width 1280 --tokens 257 --head-dim 80 --attn-variants 2,5,2,5,2,5 --iters 20
step c4 400 python bench.py --model ViT-L/14@336px --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
step c5 400 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline
