#!/bin/bash
# Row plans of the persistent GEMM at the strong split's per-rank shapes: the bit-exact
# GEMM tests, op-level times of variants 259 / 192 / 129 / 130 / 0 at 256..16 images,
# then the strong sweep with the working tree's library and with build/base's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-rows}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_gemm_rows.py "tests/test_gpu_largebatch.py::test_strong_split_shards_bitwise_vitl14" \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for b in 256 128 64 32 16; do
  timeout -k 10 300 python scripts/bench_ops.py --batch $b --ops gemm --variants 259,192,129,130,0 \
      --iters 20 > $O/ops_b$b.jsonl 2> $O/ops_b$b.err || { echo "ops b=$b failed"; tail -5 $O/ops_b$b.err; exit 1; }
done
python3 - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ops_b*.jsonl")):
    rows = [json.loads(l) for l in open(f) if l.startswith("{")]
    by = {}
    for r in rows:
        by.setdefault(r["op"], {})[r["variant"]] = r["ms"]
    print(f.split("/")[-1], {k: v for k, v in by.items()})
PY
OUT=$(basename $O)/new bash scripts/strong_sweep.sh || exit 1
OUT=$(basename $O)/base LIB=build/base/libmiclip_base.so bash scripts/strong_sweep.sh || exit 1
