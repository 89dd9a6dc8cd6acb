set -e
mkdir -p gpurun_out/stamps
for s in fc qkv out; do timeout -k 10 120 python scripts/stamps/run.py gemm --shape $s > gpurun_out/stamps/$s.json; done
timeout -k 10 120 python scripts/stamps/run.py gemm --shape fc --null > gpurun_out/stamps/fc_null.json
timeout -k 10 120 python scripts/stamps/run.py gemm --shape fc --m 65792 > gpurun_out/stamps/fc_65792.json
echo ok
