#!/bin/bash
# r04: three-deep score pipeline in the head-dim-80 two-phase attention -- bitwise + timing
# A/B against the previous build (build/prev/libmiclip_prev.so, same process), attention
# tests, C5 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04pipe3
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step ab 300 python scripts/probe/prev_vs_new.py build/prev/libmiclip_prev.so
step tests 500 $PYT tests/test_gpu_kernels.py -k "attention"
step c5 400 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline
