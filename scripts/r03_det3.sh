#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03det
mkdir -p $O
CASES=proj,proj0,fc1 WIDTH=1024 REPS=100 timeout -k 10 500 python scripts/probe/det_concurrent.py 128 > $O/det_conc2.txt 2>&1; grep -v amdgpu.ids $O/det_conc2.txt
