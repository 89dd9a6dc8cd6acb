#!/bin/bash
# r04 PMC evidence: SQ counter passes over one unsplit bench step (scripts/pmc.sh bench)
# and over the attention op (pmc.sh attn); summaries by scripts/pmc_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
rm -rf gpurun_out/pmc
bash scripts/pmc.sh bench > gpurun_out/pmc_bench.log 2>&1 || { tail -5 gpurun_out/pmc_bench.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_bench_summary.jsonl || exit 1
mkdir -p gpurun_out/pmc_bench_r04 && cp -r gpurun_out/pmc/b* gpurun_out/pmc_bench_r04/
head -c 3000 gpurun_out/pmc_bench_summary.jsonl
