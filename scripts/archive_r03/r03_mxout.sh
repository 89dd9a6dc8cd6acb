#!/bin/bash
# MX-fp8 out-projection: MX tests / parity (printed 1-cos) and the C5 whole step
# against MICLIP_MX_OUT=0 (fp16 out-proj), same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03mo
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s -k mxfp8 --timeout 200 --timeout-method thread > $O/parity.log 2>&1; rc=$?; grep "1-cos" $O/parity.log; tail -1 $O/parity.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_openclip.py tests/test_gpu_largebatch.py -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1; grep "1-cos" $O/tests.log; tail -1 $O/tests.log
bash scripts/ab_env.sh "MICLIP_MX_OUT=1" "MICLIP_MX_OUT=0" 2 --model ViT-H-14 --dtype mxfp8 --batch 512 > $O/ab.txt 2>&1; cat $O/ab.txt
