# In-kernel stamps of the four ViT-L/14 GEMM shapes (M = 32896, the benched split)
# and of the x8 attention kernel, one launch each -> gpurun_out/stamps/*.json
set -e
mkdir -p gpurun_out/stamps
for s in fc qkv out proj; do timeout -k 10 120 python scripts/stamps/run.py gemm --shape $s > gpurun_out/stamps/$s.json; done
timeout -k 10 120 python scripts/stamps/run.py attn > gpurun_out/stamps/attn.json
echo ok
