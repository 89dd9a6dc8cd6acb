#!/bin/bash
# rocprofv3 kernel statistics of the profiled (unsplit) bench step, then the
# FETCH_SIZE / WRITE_SIZE passes over gemm_fc (scripts/pmc.sh traffic; the
# traffic JSON is copied under gpurun_out so it comes back).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/rocprof" -o run \
     -- python3 bench.py --steps 5 --warmup 2 --splits 1 --no-cpu-baseline > $O/bench_prof_splits1.json 2> $O/rocprof.err \
  && echo "rocprof ok" \
  && MICLIP_TRAFFIC_SOURCE=profiles/r05/pmc_traffic bash scripts/pmc.sh traffic > $O/pmc.log 2>&1 \
  && tail -2 $O/pmc.log && cp profiles/traffic_gemm_fc.json $O/traffic_gemm_fc.json
