#!/bin/bash
# C5: MX GEMM tile-group size (MICLIP_GEMM_GROUP, default 4), interleaved, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03g
mkdir -p $O
for r in 1 2; do for g in 4 2 8 16; do
  out=$(MICLIP_GEMM_GROUP=$g timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --no-profile 2>/dev/null | tail -1)
  echo "group=$g $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("clock_ghz"))')"
done; done > $O/group.txt; cat $O/group.txt
