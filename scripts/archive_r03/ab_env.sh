#!/bin/bash
# Same-box A/B of whole-step throughput between two environment settings
# (kernel selection knobs are read once per process), interleaved R rounds.
#   bash scripts/ab_env.sh "MICLIP_ATTN=2" "MICLIP_ATTN=0" [rounds] [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
a=$1; b=$2; rounds=${3:-2}; shift 3 || true
for r in $(seq 1 "$rounds"); do
  for e in "$a" "$b"; do
    out=$(env $e timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile "$@" 2>/dev/null | tail -1) || { echo "bench failed ($e)"; exit 1; }
    echo "$e $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], "clock", d.get("clock_ghz"))')"
  done
done
