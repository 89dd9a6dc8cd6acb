#!/bin/bash
# Same-box A/B of the head-dim-80 attention (working tree vs build/abx/libmiclip_base.so)
# and of the C5 whole step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03ab
mkdir -p $O
for r in 1 2 3; do
  for L in build/abx/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
    echo "$(basename $L) $(MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ops.py --batch 256 --width 1280 --head-dim 80 --ops attention 2>/dev/null | tail -1)"
  done
done > $O/attn80_ab.txt; cat $O/attn80_ab.txt
for r in 1 2; do
  for L in build/abx/libmiclip_base.so aihab-clip_amd/miclip/libmiclip.so; do
    out=$(MICLIP_LIB=$L timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --no-profile 2>/dev/null | tail -1)
    echo "$(basename $L) $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("clock_ghz"))')"
  done
done > $O/c5_ab.txt; cat $O/c5_ab.txt
