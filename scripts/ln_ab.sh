# LayerNorm op A/B (bench_ln.py), HEAD library vs working tree, 3 interleaved rounds,
# after the LayerNorm / MX / lnfold tests
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/ln
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py tests/test_gpu_lnfold.py -x -q --timeout 120 --timeout-method thread -k "layernorm or ln" > gpurun_out/ln/t.log 2>&1; rc=$?; tail -2 gpurun_out/ln/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in build/diag/libmiclip_head.so aihab-clip_amd/miclip/libmiclip.so; do
  MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ln.py >> gpurun_out/ln/ops.jsonl || exit 1
done; done
cat gpurun_out/ln/ops.jsonl
