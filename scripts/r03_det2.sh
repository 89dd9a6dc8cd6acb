#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03det
mkdir -p $O
for args in "ViT-H-14 fp16 256 4" "ViT-L/14 mxfp8 256 4" "ViT-H-14 mxfp8 256 4"; do
  timeout -k 10 300 python scripts/probe/mx_determinism2.py $args 2>&1 | grep -v amdgpu.ids
done > $O/det_model2.txt; cat $O/det_model2.txt
