# fp16 MX quantiser (quant_mx_h8_kernel): HEAD vs 32-bit index math vs 4 chunks per
# thread (diagnostic libs), op level, 3 interleaved rounds, after the MX tests
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/quant
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py -x -q --timeout 120 --timeout-method thread > gpurun_out/quant/t.log 2>&1; rc=$?; tail -1 gpurun_out/quant/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in build/diag/libmiclip_head.so build/diag/libmiclip_q32u1.so; do
  MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ln.py > gpurun_out/quant/one.jsonl || exit 1
  grep quant_c5 gpurun_out/quant/one.jsonl >> gpurun_out/quant/ops.jsonl
done; done
cat gpurun_out/quant/ops.jsonl
