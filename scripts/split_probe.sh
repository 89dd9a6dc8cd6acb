#!/bin/bash
# Small batches: the bench's splits A/B (1/2/3 streams, interleaved) with the stream
# split floor lowered to 8 images / 2048 rows per part (build/exp/libmiclip_split.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-split2}
mkdir -p $O
for b in 32 16; do
  MICLIP_LIB=build/exp/libmiclip_split.so timeout -k 10 300 python bench.py --batch $b --steps $((2560/b)) --warmup 3 \
     --no-cpu-baseline --no-profile --ab-splits > $O/bs$b.json 2> $O/bs$b.err || { tail -5 $O/bs$b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bs$b.json').read().strip().splitlines()[-1]); print($b, d['value'], d['splits_ab_img_s'])"
done
