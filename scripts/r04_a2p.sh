#!/bin/bash
# r04: two-phase one-head-per-workgroup attention (N > 320) -- tests, C4 parity, op A/B, C4 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04a2p
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 2 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 500 $PYT tests/test_gpu_kernels.py -k "attention"
step parity 600 $PYT tests/test_gpu_parity.py tests/test_gpu_largebatch.py -k "336 or vitl14_336 or c4"
step ops 300 python scripts/bench_ops.py --ops attention --batch 128 --width 1024 --tokens 577 --attn-variants 1,3,1,3,1,3 --iters 20
step c4 400 python bench.py --model ViT-L/14@336px --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
