#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04a80b
mkdir -p "$out"
timeout -k 10 300 python scripts/bench_ops.py --ops attention --batch 256 --width 1280 --head-dim 80 --tokens 257 --attn-variants 1,2,1,2,1,2 --iters 30 > $out/ops.log 2>&1; rc=$?; grep '"op"' $out/ops.log; exit $rc
