# Persistent GEMM start-stagger diagnostic (kGemmStagger on variant 259): op level,
# 3 interleaved rounds of no stagger / 4 / 8 / 16 us -> gpurun_out/gstag/
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/gstag
for r in 1 2 3; do
  timeout -k 10 200 python scripts/bench_ops.py --ops gemm --only qkv,fc,proj,out --variants 259,8650755,259s,33816835 >> gpurun_out/gstag/ops.jsonl || exit 1
done
cat gpurun_out/gstag/ops.jsonl
