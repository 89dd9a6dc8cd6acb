# gemm_group() 8 vs 4 (HEAD): GEMM tests, then the model A/B, 3 interleaved rounds
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/gm8
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_lnfold.py -x -q --timeout 120 --timeout-method thread -k "gemm or fold" > gpurun_out/gm8/t.log 2>&1; rc=$?; tail -1 gpurun_out/gm8/t.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh build/diag/libmiclip_head.so 3 | tee gpurun_out/gm8/model_ab.txt
