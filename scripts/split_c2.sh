#!/bin/bash
# C2 (ViT-B/32 bf16 bs=256) and C4 splits A/B with the stream-split row floor lowered.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-split_c2}
mkdir -p $O
MICLIP_LIB=build/exp/libmiclip_split.so timeout -k 10 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 20 --warmup 3 --no-cpu-baseline --no-profile --ab-splits > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['splits_ab_img_s'])"
for b in 48 96; do
MICLIP_LIB=build/exp/libmiclip_split.so timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 3 --no-cpu-baseline --no-profile --ab-splits > $O/l14_$b.json 2> $O/l14_$b.err || { tail -5 $O/l14_$b.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/l14_$b.json').read().strip().splitlines()[-1]); print('l14 $b', d['value'], d['splits_ab_img_s'])"
done
