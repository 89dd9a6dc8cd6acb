#!/bin/bash
# Same-box A/B of whole-step throughput: bench.py with the working tree's library
# against a baseline library (scripts/build_base_lib.sh), interleaved R rounds.
#   bash scripts/ab_bench.sh build/ab/libmiclip_HEAD.so [rounds] [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
base=$1; rounds=${2:-2}; shift 2 || true
for r in $(seq 1 "$rounds"); do
  for L in "$base" aihab-clip_amd/miclip/libmiclip.so; do
    out=$(MICLIP_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile "$@" 2>/dev/null | tail -1) || { echo "bench failed ($L)"; exit 1; }
    echo "$L $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], "clock", d.get("clock_ghz"))')"
  done
done
