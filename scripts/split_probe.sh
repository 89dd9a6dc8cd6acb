#!/bin/bash
# Small batches: the bench's splits A/B (1/2/3 streams, interleaved) with the
# stream-split row floor lowered (build/exp/libmiclip_split.so, MICLIP_SPLIT_ROWS=2048),
# the strong sweep of the working tree, and attention variants at 16/32 images.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-split}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_rows.py \
    "tests/test_gpu_largebatch.py::test_strong_split_shards_bitwise_vitl14" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
OUT=$(basename $O)/splits LIB=build/exp/libmiclip_split.so BATCHES="128 64 32 16" EXTRA="--ab-splits --no-profile" bash scripts/strong_sweep.sh || exit 1
OUT=$(basename $O)/new bash scripts/strong_sweep.sh || exit 1
for b in 32 16; do
  timeout -k 10 120 python scripts/bench_ops.py --batch $b --ops attention --attn-variants 8,2,0,8,2,0 > $O/attn_b$b.jsonl 2> $O/attn_b$b.err || { tail -3 $O/attn_b$b.err; exit 1; }
  python3 -c "
import json; r=[json.loads(l) for l in open('$O/attn_b$b.jsonl') if l.startswith('{')]
print($b, [(x['variant'], x['ms']) for x in r])"
done
