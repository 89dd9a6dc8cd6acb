# GPU A/B step: GEMM correctness subset, op-level and whole-step A/B against build/diag/libmiclip_head.so
set -o pipefail
export MICLIP_QUIET=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_lnfold.py tests/test_gpu_mx.py -x -q --timeout 120 --timeout-method thread -k "gemm or fold or mx" > gpurun_out/t_gemm.log 2>&1; rc=$?; tail -2 gpurun_out/t_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_parity.log 2>&1; rc=$?; tail -2 gpurun_out/t_parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_ops.sh build/diag/libmiclip_head.so 3 || exit 1
bash scripts/ab_bench.sh build/diag/libmiclip_head.so 3 || exit 1
