#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04dist
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 2 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step tests 400 $PYT tests/test_gpu_distributed.py tests/test_gpu_drivers.py
step bench 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 5
