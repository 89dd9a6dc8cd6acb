#!/bin/bash
# Hardware evidence for the current tree -> gpurun_out/evidence/:
#   pmc/b1..b3  per-kernel SQ counters over one unsplit bench step (scripts/pmc.sh bench)
#   pmc/fetch, pmc/write  FETCH_SIZE / WRITE_SIZE passes (scripts/pmc.sh traffic)
#   stats/      rocprofv3 --kernel-trace --stats of bench.py --splits 1 (the profiled-step form)
#   bench.json  the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/evidence
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/stats -o run -- python3 bench.py --splits 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/stats.json 2> $O/stats.err || { tail -5 $O/stats.err; exit 1; }
bash scripts/pmc.sh bench > $O/pmc_bench.log 2>&1 || { tail -5 $O/pmc_bench.log; exit 1; }
bash scripts/pmc.sh traffic > $O/pmc_traffic.log 2>&1 || { tail -5 $O/pmc_traffic.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc > $O/pmc_summary.txt 2>&1
mv gpurun_out/pmc $O/pmc
echo ok
