#!/bin/bash
# SURVEY §8e's strong split on one GPU: the per-rank workload of a global 256 split
# G ways (256/128/64/32 images per GPU) plus the reference's own batch 16
# (configs/cs.yaml:15), one bench line each -> gpurun_out/${OUT:-strong}/bs<b>.json.
# Steps scale with 1/b so every timed region is ~0.4 s of GPU work.
#   OUT=name BATCHES="256 128 64 32 16" EXTRA="--ab-splits" [LIB=other.so] bash scripts/strong_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1 MICLIP_AB_BUILD=1
O=gpurun_out/${OUT:-strong}
mkdir -p $O
for b in ${BATCHES:-256 128 64 32 16}; do
  s=$(( 2560 / b )); [ $s -lt 10 ] && s=10
  ${LIB:+env MICLIP_LIB=$LIB} timeout -k 10 300 python bench.py --scaling strong --batch $b --steps $s --warmup 3 \
      --no-cpu-baseline ${EXTRA:-} > $O/bs$b.json 2> $O/bs$b.err || { echo "bench bs=$b failed"; tail -5 $O/bs$b.err; exit 1; }
  python3 - "$O/bs$b.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(d["config"]["images_per_gpu"], d["value"], "img/s clk", d.get("clock_ghz"),
      "splits", d["config"]["splits"], d.get("splits_ab_img_s", ""),
      " ".join(f"{n}={v['ms']:.3f}" for n, v in k.items() if v["ms"] > 0.02))
EOF
done
