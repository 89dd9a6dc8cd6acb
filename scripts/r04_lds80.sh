#!/bin/bash
# r04: conflict-free LDS layouts (head-dim-80 K/V images; a MX LayerNorm gamma/beta
# reorder was measured in the same run and dropped) -- bitwise + timing A/B against the
# previous build (build/prev/libmiclip_prev.so, a copy of the library before the change,
# same process), attention / LayerNorm / MX tests, C5 parity, C5 bench, PMC of one C5 step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04lds
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step ab 300 python scripts/probe/prev_vs_new.py build/prev/libmiclip_prev.so
step tests 500 $PYT tests/test_gpu_kernels.py tests/test_gpu_mx.py -k "attention or layernorm"
step parity 600 $PYT tests/test_gpu_openclip.py tests/test_gpu_largebatch.py tests/test_gpu_parity.py -k "openclip or vith14 or H-14"
step c5 400 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline
step pmc 600 bash scripts/r04_pmc_c5.sh
