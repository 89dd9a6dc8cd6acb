set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/gstag
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/gstag/t.log 2>&1; rc=$?; tail -1 gpurun_out/gstag/t.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh build/diag/libmiclip_head.so 3 | tee gpurun_out/gstag/model_ab.txt
