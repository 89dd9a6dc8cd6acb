#!/bin/bash
# r04: C2 small-launch LayerNorm (8 rows per workgroup) + attention variants at N = 50
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r04c2b}
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 600 $PYT tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_largebatch.py tests/test_gpu_lnfold.py
step ops 300 python scripts/bench_ops.py --ops attention --batch 256 --width 768 --tokens 50 --attn-variants 0,1,2,0,1,2 --iters 20
step bench 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline
