#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03det
mkdir -p $O
REPS=8 timeout -k 10 200 python scripts/probe/det_ops.py 128 > $O/det_ops.txt 2>&1; cat $O/det_ops.txt | grep -v amdgpu.ids
timeout -k 10 300 python scripts/probe/mx_determinism2.py ViT-H-14 mxfp8 512 4 > $O/det_model.txt 2>&1; cat $O/det_model.txt | grep -v amdgpu.ids
