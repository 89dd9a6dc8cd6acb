#!/bin/bash
# Small-batch diagnostics: interleaved op-level row plans (rows_ops.py), eager vs
# HIP-graph encode at 16/32/64 images, and a kernel trace of the bs=32 bench step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-small}
mkdir -p $O
timeout -k 10 400 python scripts/rows_ops.py --c2 > $O/rows_ops.jsonl 2> $O/rows_ops.err || { tail -5 $O/rows_ops.err; exit 1; }
for b in 16 32 64; do
  timeout -k 10 200 python scripts/graph_probe.py $b > $O/graph_b$b.txt 2>&1 || { tail -5 $O/graph_b$b.txt; exit 1; }
  tail -3 $O/graph_b$b.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace32 -o trace -- python3 bench.py --batch 32 --steps 20 --warmup 3 --no-cpu-baseline --no-profile > $O/trace32.json 2> $O/trace32.err || { tail -5 $O/trace32.err; exit 1; }
echo ok
