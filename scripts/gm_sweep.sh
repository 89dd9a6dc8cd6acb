# Persistent GEMM tile-group height (gm, variant + 1000 gm) sweep at the ViT-L/14 shapes,
# op level, 3 interleaved rounds -> gpurun_out/gm/
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/gm
for r in 1 2 3; do
  timeout -k 10 200 python scripts/bench_ops.py --ops gemm --only fc,qkv,proj,out --variants 8259,4259,2259,16259,4259,8259 >> gpurun_out/gm/ops.jsonl || exit 1
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/gm/ops.jsonl"):
    j = json.loads(l); d[(j["op"], j["variant"])].append(j["ms"])
for k in sorted(d): print(k, sorted(d[k]))
PY
