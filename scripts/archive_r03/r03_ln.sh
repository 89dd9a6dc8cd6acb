#!/bin/bash
# LayerNorm (fp16 stream, MX output) with gamma/beta in LDS: tests + same-box C5 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03ln
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_largebatch.py tests/test_gpu_openclip.py -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; grep "1-cos" $O/tests.log; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 200 --timeout-method thread > $O/parity.log 2>&1; rc=$?; grep "1-cos" $O/parity.log | head -30; tail -1 $O/parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for L in build/abx/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
  out=$(MICLIP_LIB=$L timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --no-profile 2>/dev/null | tail -1)
  echo "$(basename $L) $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("clock_ghz"))')"
done; done > $O/c5_ab.txt; cat $O/c5_ab.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o ln -- python3 $GRAFT_REPO_ROOT/bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
