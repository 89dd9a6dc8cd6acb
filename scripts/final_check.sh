#!/bin/bash
# Final-tree check: the full GPU suite, smoke() and the default bench line -> gpurun_out/final_check/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1 TMPDIR=/tmp
O=gpurun_out/final_check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  && tail -1 $O/pytest_gpu.log \
  && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  && tail -1 $O/smoke.log \
  && timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err \
  && python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_mfma_frac'], d['clock_ghz'])"
