#!/bin/bash
# GPU test subset (or the whole suite with no args), each run under its own limit.
#   OUT=name bash scripts/gpu_tests.sh [pytest args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MICLIP_QUIET=1
O=gpurun_out/${OUT:-tests}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "${@:-tests}" > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
exit $rc
