# MX LayerNorm rows per workgroup (diagnostic libs: 8 / 16 vs the default 32), op level,
# 3 interleaved rounds -> gpurun_out/lnmx/
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/lnmx
for r in 1 2 3; do for L in aihab-clip_amd/miclip/libmiclip.so build/diag/libmiclip_lnmx8.so build/diag/libmiclip_lnmx16.so; do
  MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ln.py > gpurun_out/lnmx/one.jsonl || exit 1
  grep mx_c5 gpurun_out/lnmx/one.jsonl >> gpurun_out/lnmx/ops.jsonl
done; done
cat gpurun_out/lnmx/ops.jsonl
