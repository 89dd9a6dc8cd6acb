#!/bin/bash
# Same-box A/B of an experiment library (EXP, default build/exp/libmiclip_dma.so) against
# the working tree's: its GEMM tests, op-level GEMM times (rows_ops.py at 256 / 32
# images, interleaved 3 rounds), then R interleaved rounds of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1 MICLIP_AB_BUILD=1
EXP=${EXP:-build/exp/libmiclip_dma.so}
O=gpurun_out/${OUT:-lib_ab}
mkdir -p $O
MICLIP_LIB=$EXP timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_gemm_rows.py tests/test_gpu_lnfold.py tests/test_gpu_splitk.py > $O/pytest_exp.log 2>&1 || { tail -30 $O/pytest_exp.log; exit 1; }
tail -1 $O/pytest_exp.log
for r in 1 2 3; do
  for L in aihab-clip_amd/miclip/libmiclip.so $EXP; do
    n=$(basename $L .so)
    MICLIP_LIB=$L timeout -k 10 200 python scripts/rows_ops.py --batches 256,32 --variants 0 --rounds 1 > $O/ops_${r}_$n.jsonl 2>/dev/null || exit 1
    echo "$r $n $(python3 -c "
import json; print(' '.join(f\"{d['shape']}={d['ms']}\" for d in map(json.loads, open('$O/ops_${r}_$n.jsonl'))))")"
  done
done
for r in $(seq 1 ${R:-3}); do
  for L in aihab-clip_amd/miclip/libmiclip.so $EXP; do
    n=$(basename $L .so)
    MICLIP_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${r}_$n.json 2> $O/b_${r}_$n.err || { echo "bench failed ($L)"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${r}_$n.json').read().strip().splitlines()[-1]); k=d.get('kernels',{})
print('$n', d['value'], 'clk', d.get('clock_ghz'), ' '.join(f'{n}={v[\"ms\"]:.3f}' for n,v in k.items() if v['ms']>0.1))"
  done
done
