#!/bin/bash
# Same-box A/B step: GPU tests (args: pytest paths), then R interleaved rounds of
# the default bench against build/base/libmiclip_base.so (scripts/build_base_lib.sh
# output copied there: build/ab is not uploaded).
#   OUT=name R=3 bash scripts/ab_step.sh tests/test_x.py ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1 MICLIP_AB_BUILD=1
O=gpurun_out/${OUT:-ab}
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" > $O/pytest_gpu.log 2>&1
  rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${R:-3}); do
  for L in build/base/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
    MICLIP_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${r}_$(basename $L .so).json 2> $O/b_${r}_$(basename $L .so).err || { echo "bench failed ($L)"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${r}_$(basename $L .so).json').read().strip().splitlines()[-1])
k=d.get('kernels',{})
print('$L'.split('/')[-1], d['value'], 'clk', d.get('clock_ghz'), ' '.join(f'{n}={v[\"ms\"]:.3f}' for n,v in k.items() if v['ms']>0.1))"
  done
done
