#!/bin/bash
# Parity with printed 1-cos values, then one bench line per secondary BASELINE config
# (C2 ViT-B/32 bf16, C4 ViT-L/14@336px fp16, C5 ViT-H-14 MX-fp8 bs=512) -> gpurun_out/${OUT:-configs}/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-configs}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 120 --timeout-method thread > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline'] or {}
print('$2', d['value'], 'img/s', 'path_frac', d['path_mfma_frac'], 'clk', d['clock_ghz'], r.get('clock_ghz_per_xcd'), 'rej', r.get('clock_rejected_per_xcd'))"; }
timeout -k 10 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 30 --warmup 3 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
summ $O/c2.json C2
timeout -k 10 300 python bench.py --model ViT-L/14@336px --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
summ $O/c4.json C4
timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 1
summ $O/c5.json C5
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/c3.json 2> $O/c3.err || exit 1
summ $O/c3.json C3
echo ok
