#!/bin/bash
# MX-fp8 path after the tanh-form GELU in the c_fc epilogue: op tests, model
# parity (printed 1-cos), open_clip surface, large batch, and the C5 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03mx
mkdir -p $O
timeout -k 10 200 python scripts/probe/mx_epi.py > $O/mx_epi.jsonl 2>&1; grep fc $O/mx_epi.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_openclip.py tests/test_gpu_largebatch.py -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s -k mxfp8 --timeout 200 --timeout-method thread > $O/parity.log 2>&1; rc=$?; grep -i "1-cos\|1−cos\|cos" $O/parity.log | head -20; tail -2 $O/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err \
  && python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], d['path_mfma_frac'], d.get('clock_ghz')); [print(' ',k,v) for k,v in d['kernels'].items()]"
