#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03det
mkdir -p $O
{
CASES=proj,qkv,fc WIDTH=1024 REPS=100 timeout -k 10 300 python scripts/probe/det_concurrent.py 128 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python scripts/probe/mx_determinism2.py ViT-L/14 mxfp8 256 6 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python scripts/probe/mx_determinism2.py ViT-H-14 mxfp8 512 4 2>&1 | grep -v amdgpu.ids
} > $O/det_fixed.txt; cat $O/det_fixed.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_largebatch.py tests/test_gpu_openclip.py -x -q -s --timeout 200 --timeout-method thread > $O/tests_fixed.log 2>&1; tail -3 $O/tests_fixed.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k "dh80 or attention_q0" -x -q --timeout 100 --timeout-method thread > $O/attn80.log 2>&1; tail -2 $O/attn80.log
timeout -k 10 120 python scripts/bench_ops.py --batch 256 --width 1280 --head-dim 80 --ops attention > $O/attn80_ops.jsonl 2>&1; grep attention $O/attn80_ops.jsonl
