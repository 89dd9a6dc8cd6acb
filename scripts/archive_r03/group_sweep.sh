# whole-step throughput over the persistent GEMM's tile-row group (MICLIP_GEMM_GROUP), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do for g in 4 2 8 16; do
  out=$(MICLIP_GEMM_GROUP=$g MICLIP_QUIET=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1) || { echo fail; exit 1; }
  echo "r$r group=$g $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); k=d["kernels"]; print(d["value"], d["ms_per_step"], "fc", k["gemm_fc"]["ms"], "qkv", k["gemm_qkv"]["ms"], "proj", k["gemm_proj"]["ms"], "out", k["gemm_out"]["ms"])')"
done; done
