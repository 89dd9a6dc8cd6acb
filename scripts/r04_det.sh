#!/bin/bash
# r04: run-to-run determinism with the persistent MX GEMM, 192-row tiles and split-K CLS GEMMs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04det
mkdir -p "$out"
for args in "ViT-H-14 mxfp8 512 4" "ViT-B/32 bf16 256 6" "ViT-L/14 fp16 256 4"; do
  timeout -k 10 300 python scripts/probe/mx_determinism2.py $args >> $out/det.txt 2>&1 || { tail -5 $out/det.txt; exit 1; }
done
grep -v amdgpu.ids $out/det.txt
