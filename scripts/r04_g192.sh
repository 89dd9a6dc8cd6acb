#!/bin/bash
# r04: 192-row GEMM tiles -- bit-exactness, C2 parity / large batch, C2 A/B (auto vs 259)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r04g192}
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 500 $PYT tests/test_gpu_gemm192.py tests/test_gpu_kernels.py -k "gemm"
step parity 500 $PYT tests/test_gpu_parity.py tests/test_gpu_largebatch.py -k "vitb32 or bf16"
step ab 400 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline --ab-gemm 0:0,259:259,0:259,259:0
