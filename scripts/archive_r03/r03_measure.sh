#!/bin/bash
# r03 re-entry measurement: default bench line, op-level and whole-step A/B of the
# opt-in ping-pong GEMM (MICLIP_GEMM=400) and streamed attention (MICLIP_ATTN=9).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-profile --no-cpu-baseline > $O/bench.json 2> $O/bench.err \
  && tail -c 300 $O/bench.json && echo \
  && timeout -k 10 120 python -u -m pytest tests/test_gpu_gemm_pp.py -x -q --timeout 60 --timeout-method thread > $O/pp_tests.log 2>&1 \
  && tail -1 $O/pp_tests.log \
  && timeout -k 10 200 python scripts/bench_ops.py --batch 128 --ops gemm --variants 0,400,0,400,402 > $O/ops_gemm.jsonl 2>&1 \
  && cat $O/ops_gemm.jsonl \
  && timeout -k 10 120 python scripts/bench_ops.py --batch 128 --ops attention > $O/ops_attn.jsonl 2>&1 \
  && cat $O/ops_attn.jsonl \
  && bash scripts/ab_env.sh "MICLIP_GEMM=400" "MICLIP_GEMM=0" 2 > $O/ab_gemm.txt 2>&1 \
  && cat $O/ab_gemm.txt \
  && bash scripts/ab_env.sh "MICLIP_ATTN=9" "MICLIP_ATTN=0" 2 > $O/ab_attn.txt 2>&1 \
  && cat $O/ab_attn.txt
