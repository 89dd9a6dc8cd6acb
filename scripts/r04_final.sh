#!/bin/bash
# r04 evidence in one GPU call (outputs gpurun_out/r04final/, kept ones copied to
# profiles/r04/): the full GPU suite, smoke(), the default bench line, rocprofv3
# kernel stats of the profiled (unsplit) bench step, the FETCH_SIZE / WRITE_SIZE
# passes over gemm_fc, and one bench line per secondary config (C2, C4, C5).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-r04final}
mkdir -p $O/configs
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  && tail -1 $O/pytest_gpu.log \
  && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  && tail -1 $O/smoke.log \
  && timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err \
  && tail -c 300 $O/bench.json \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/rocprof" -o run \
       -- python3 bench.py --steps 5 --warmup 2 --splits 1 --no-cpu-baseline > $O/bench_prof_splits1.json 2> $O/rocprof.err \
  && echo "rocprof ok" \
  && MICLIP_TRAFFIC_SOURCE=profiles/r04/pmc_traffic bash scripts/pmc.sh traffic > $O/pmc.log 2>&1 \
  && tail -2 $O/pmc.log \
  && timeout -k 10 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > $O/configs/c2.json 2> $O/configs/c2.err \
  && timeout -k 10 300 python bench.py --model ViT-L/14@336px --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > $O/configs/c4.json 2> $O/configs/c4.err \
  && timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > $O/configs/c5.json 2> $O/configs/c5.err \
  && echo "configs ok" \
  && timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --ab-splits > $O/configs/c3_ab_splits.json 2>&1 \
  && echo "ab splits ok"
