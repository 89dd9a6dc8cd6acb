# whole-step throughput at 2 / 3 / 4 stream splits of the bs=256 batch, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do for sp in 2 3 4; do
  out=$(MICLIP_QUIET=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --splits $sp 2>/dev/null | tail -1) || { echo fail; exit 1; }
  echo "r$r splits=$sp $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["config"]["splits"])')"
done; done
