#!/bin/bash
# Round-3 evidence in one GPU call: final_profile.sh (GPU suite, smoke, bench line,
# rocprofv3 stats, FETCH/WRITE passes) then the per-kernel PMC passes of one step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r03}
bash scripts/final_profile.sh "$tag" && timeout -k 10 300 bash scripts/pmc.sh bench > gpurun_out/final/pmc_bench.log 2>&1 \
  && tail -3 gpurun_out/final/pmc_bench.log
