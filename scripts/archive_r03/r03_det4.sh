#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03det
mkdir -p $O
{
echo "== CLS_LAST=0"; MICLIP_CLS_LAST=0 timeout -k 10 300 python scripts/probe/mx_determinism2.py ViT-L/14 mxfp8 256 4 2>&1 | grep -v amdgpu.ids
echo "== bs 64"; timeout -k 10 300 python scripts/probe/mx_determinism2.py ViT-L/14 mxfp8 64 4 2>&1 | grep -v amdgpu.ids
echo "== ViT-B/32 mx bs 512"; timeout -k 10 300 python scripts/probe/mx_determinism2.py ViT-B/32 mxfp8 512 4 2>&1 | grep -v amdgpu.ids
} > $O/det_model4.txt; cat $O/det_model4.txt
