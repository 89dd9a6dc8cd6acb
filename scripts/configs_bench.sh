# Parity with printed 1-cos values, then one bench line per secondary BASELINE config
# (C2 ViT-B/32 bf16, C4 ViT-L/14@336 fp16, C5 ViT-H-14 MX-fp8 bs=512) -> gpurun_out/configs/
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/configs
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/configs/parity.log 2>&1; rc=$?; tail -2 gpurun_out/configs/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/configs/c2.json 2> gpurun_out/configs/c2.err || exit 1
timeout -k 10 300 python bench.py --model ViT-L/14@336px --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/configs/c4.json 2> gpurun_out/configs/c4.err || exit 1
timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/configs/c5.json 2> gpurun_out/configs/c5.err || exit 1
echo ok
