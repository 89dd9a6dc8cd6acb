#!/bin/bash
# r04: two-phase head-dim-80 attention -- kernel tests, open_clip / C5 parity, op A/B, C5 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r04a80}
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 500 $PYT tests/test_gpu_kernels.py -k "attention"
step parity 500 $PYT tests/test_gpu_openclip.py tests/test_gpu_largebatch.py -k "vith or mx or MX"
step ops 300 python scripts/bench_ops.py --ops attention --batch 256 --width 1280 --head-dim 80 --tokens 257 --attn-variants 1,2,1,2,1,2 --iters 20
step c5 400 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline
