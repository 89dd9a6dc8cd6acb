#!/bin/bash
# r04 PMC of one unsplit C5 step (ViT-H-14 MX-fp8 bs=512: attention80s_kernel, MX GEMMs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
rm -rf gpurun_out/pmc
PMC_BENCH_ARGS="--model ViT-H-14 --dtype mxfp8 --batch 512" bash scripts/pmc.sh bench > gpurun_out/pmc_c5.log 2>&1 || { tail -5 gpurun_out/pmc_c5.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_c5_summary.jsonl || exit 1
mkdir -p gpurun_out/pmc_c5_r04 && cp -r gpurun_out/pmc/b* gpurun_out/pmc_c5_r04/
grep -E "attention|gemm256s_mx|layernorm" gpurun_out/pmc_c5_summary.jsonl | cut -c1-400
