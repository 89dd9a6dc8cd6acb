#!/bin/bash
# Same-box interleaved A/B of the GEMM ops (bench_ops.py) and the whole step
# (ab_bench.sh): the working tree's library against a baseline library.
#   bash scripts/ab_ops.sh build/ab/libmiclip_HEAD.so [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
base=$1; rounds=${2:-3}
mkdir -p gpurun_out/ab
for r in $(seq 1 "$rounds"); do
  for L in "$base" aihab-clip_amd/miclip/libmiclip.so; do
    tag=$(basename "$L" .so)
    MICLIP_LIB=$L timeout -k 10 200 python scripts/bench_ops.py --ops gemm --variants 0 \
      > gpurun_out/ab/ops_${tag}_$r.jsonl 2>/dev/null || { echo "ops failed ($L)"; exit 1; }
    echo "$tag r$r $(python3 -c 'import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d.get("name",d.get("op")), d.get("ms"), end="; ")' gpurun_out/ab/ops_${tag}_$r.jsonl)"
  done
done
