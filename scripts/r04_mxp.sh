#!/bin/bash
# r04: persistent MX GEMM -- bit-exactness tests, MX parity tests, C5 A/B (one-tile vs persistent)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r04mxp}
mkdir -p "$out"
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step tests 500 $PYT tests/test_gpu_mx_persistent.py tests/test_gpu_mx.py
step parity 500 $PYT tests/test_gpu_openclip.py tests/test_gpu_largebatch.py -k "mx or MX or vith"
step ab 500 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --ab-gemm 0:0:1,0:0:2
