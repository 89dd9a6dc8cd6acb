#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03mq
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_largebatch.py -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1; grep "1-cos" $O/tests.log; tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s -k mxfp8 --timeout 200 --timeout-method thread > $O/parity.log 2>&1; grep "1-cos" $O/parity.log; tail -1 $O/parity.log
for r in 1 2; do for L in build/abx/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
  echo "$(basename $L) $(MICLIP_LIB=$L timeout -k 10 200 python scripts/probe/mx_epi.py 2>/dev/null | grep qkv | grep '"store"' | head -1)"
done; done > $O/qkv_ab.txt; cat $O/qkv_ab.txt
for r in 1 2; do for L in build/abx/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
  out=$(MICLIP_LIB=$L timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --no-profile 2>/dev/null | tail -1)
  echo "$(basename $L) $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("clock_ghz"))')"
done; done > $O/c5_ab.txt; cat $O/c5_ab.txt
