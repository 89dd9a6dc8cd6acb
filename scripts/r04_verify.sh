#!/bin/bash
# Round-end check of the committed tree in one GPU call: the full GPU suite,
# smoke(), and the default bench line (outputs under gpurun_out/${OUT}).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-r04verify}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  && tail -1 $O/pytest_gpu.log \
  && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  && tail -1 $O/smoke.log \
  && timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err \
  && tail -c 400 $O/bench.json
