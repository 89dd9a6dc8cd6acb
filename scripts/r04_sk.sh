#!/bin/bash
# r04: split-K GEMMs of the CLS-only last block -- model parity / invariance tests, C2 + headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r04sk}
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 700 $PYT tests/test_gpu_parity.py tests/test_gpu_largebatch.py tests/test_gpu_openclip.py tests/test_gpu_drivers.py
step c2 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline
step l14 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
