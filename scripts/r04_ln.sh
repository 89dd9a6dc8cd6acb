#!/bin/bash
# r04: LayerNorm row-pair prefetch (32-row workgroups) -- LayerNorm / MX / fold tests,
# C5 parity, C5 bench (MX LayerNorm = the 32-row path at ViT-H/14 bs=512)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04ln
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 2 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 500 $PYT tests/test_gpu_kernels.py tests/test_gpu_mx.py tests/test_gpu_lnfold.py -k "layernorm or ln_"
step parity 600 $PYT tests/test_gpu_openclip.py tests/test_gpu_largebatch.py -k "openclip or vith14 or H-14"
step c5 400 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline
step c5b 400 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline
