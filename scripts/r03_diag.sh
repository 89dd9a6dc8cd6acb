#!/bin/bash
# GEMM main-loop diagnosis (DMA-skipping variants) and C2 shape options.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 200 python scripts/bench_ops.py --batch 128 --ops gemm --only fc,proj --variants 0,259d,259e,0,259d,259e > $O/diag.jsonl 2>&1 \
  && cat $O/diag.jsonl \
  && timeout -k 10 200 python scripts/bench_ops.py --batch 256 --width 768 --tokens 50 --ops gemm,attention --variants 0,2,400,128,0 > $O/c2_ops.jsonl 2>&1 \
  && cat $O/c2_ops.jsonl
