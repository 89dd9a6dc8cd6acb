#!/bin/bash
# r04: rocprofv3 kernel statistics of the secondary configs' bench runs (C2, C4, C5),
# one rocprofv3 run each (kernel trace + stats only), unsplit (--splits 1) so that no
# kernel shares the GPU with the other stream's and the durations are per-kernel times;
# summaries under gpurun_out/r04profc/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/r04profc
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/$name" -o run \
    -- python3 bench.py "$@" --steps 5 --warmup 2 --splits 1 --no-cpu-baseline > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run c2 --model ViT-B/32 --dtype bf16
run c4 --model ViT-L/14@336px --dtype fp16
run c5 --model ViT-H-14 --dtype mxfp8 --batch 512
