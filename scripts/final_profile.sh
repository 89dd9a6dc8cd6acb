#!/bin/bash
# End-of-round evidence in one GPU call: the full GPU suite, smoke(), the default
# bench line, rocprofv3 kernel stats of the profiled (unsplit) bench step and the
# FETCH_SIZE / WRITE_SIZE passes over gemm_fc. Outputs under gpurun_out/final/
# (copy what is kept into profiles/<round>/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/final
mkdir -p $O
tag=${1:-r02b}
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  && tail -1 $O/pytest_gpu.log \
  && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  && tail -1 $O/smoke.log \
  && timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err \
  && tail -c 400 $O/bench.json \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/rocprof" -o run \
       -- python3 bench.py --steps 5 --warmup 2 --splits 1 --no-cpu-baseline > $O/bench_prof_splits1.json 2> $O/rocprof.err \
  && echo "rocprof ok" \
  && MICLIP_TRAFFIC_SOURCE=profiles/$tag/pmc_traffic bash scripts/pmc.sh traffic > $O/pmc.log 2>&1 \
  && tail -2 $O/pmc.log
