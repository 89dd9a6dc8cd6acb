#!/bin/bash
# r04 PMC of one unsplit C4 step (ViT-L/14@336px, N = 577: attention_kernel<64> on 16 waves)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
rm -rf gpurun_out/pmc
PMC_BENCH_ARGS="--model ViT-L/14@336px" bash scripts/pmc.sh bench > gpurun_out/pmc_c4.log 2>&1 || { tail -5 gpurun_out/pmc_c4.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_c4_summary.jsonl || exit 1
mkdir -p gpurun_out/pmc_c4_r04 && cp -r gpurun_out/pmc/b* gpurun_out/pmc_c4_r04/
grep attention gpurun_out/pmc_c4_summary.jsonl
