#!/bin/bash
# Attention change: kernel tests + parity, op-level x8 times (new vs build/base, 3
# interleaved rounds), then the same-box step A/B (scripts/ab_step.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1 MICLIP_AB_BUILD=1
O=gpurun_out/${OUT:-attn}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_parity.py > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
  for L in build/base/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
    MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ops.py --ops attention --attn-variants 8 --iters 20 > $O/op_${r}_$(basename $L .so).jsonl 2>/dev/null || exit 1
    echo "$r $(basename $L .so) $(grep -o '"ms": [0-9.]*' $O/op_${r}_$(basename $L .so).jsonl)"
  done
done
OUT=$(basename $O)/step R=3 bash scripts/ab_step.sh
