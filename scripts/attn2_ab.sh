#!/bin/bash
# Shift-softmax in the N = 577 one-head and head-dim-80 kernels: kernel / parity /
# large-batch / open_clip tests, op-level A/B (new vs build/base, 3 interleaved rounds)
# at C4's N = 577 and C5's head dim 80, then C4 and C5 step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1 MICLIP_AB_BUILD=1
O=gpurun_out/${OUT:-attn2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
   tests/test_gpu_parity.py tests/test_gpu_largebatch.py tests/test_gpu_openclip.py > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
  for L in build/base/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
    n=$(basename $L .so)
    MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ops.py --ops attention --attn-variants 0 --tokens 577 --iters 10 > $O/op577_${r}_$n.jsonl 2>/dev/null || exit 1
    MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ops.py --ops attention --attn-variants 0 --head-dim 80 --width 1280 --batch 512 --iters 10 > $O/op80_${r}_$n.jsonl 2>/dev/null || exit 1
    echo "$r $n 577: $(grep -o '"ms": [0-9.]*' $O/op577_${r}_$n.jsonl) dh80: $(grep -o '"ms": [0-9.]*' $O/op80_${r}_$n.jsonl)"
  done
done
for r in 1 2; do
  for L in build/base/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
    n=$(basename $L .so)
    MICLIP_LIB=$L timeout -k 10 300 python bench.py --model ViT-L/14@336px --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_${r}_$n.json 2>/dev/null || exit 1
    MICLIP_LIB=$L timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_${r}_$n.json 2>/dev/null || exit 1
    python3 -c "
import json
for c in ('c4','c5'):
    d=json.loads(open('$O/'+c+'_${r}_$n.json').read().strip().splitlines()[-1])
    print('$r $n', c, d['value'], 'clk', d['clock_ghz'], 'attn', d['kernels']['attention']['ms'])"
  done
done
