#!/bin/bash
# Prices of step components inside the two-stream bench step: R interleaved rounds
# of bench.py with the product library and each timing-diagnostic library
# (make diag: no vision attention / no large ln_stats launches; outputs meaningless).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-diag}
mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for L in aihab-clip_amd/miclip/libmiclip.so build/diag/libmiclip_noattn.so build/diag/libmiclip_nolns.so ${EXTRA_LIBS:-}; do
    n=$(basename $L .so)
    MICLIP_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${r}_$n.json 2> $O/b_${r}_$n.err || { echo "bench failed ($L)"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${r}_$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], 'clk', d.get('clock_ghz'))"
  done
done
