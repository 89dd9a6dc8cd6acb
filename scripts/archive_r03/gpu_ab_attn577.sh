# one-head-per-workgroup attention (N = 577, C4): correctness, op and C4 whole-step A/B
set -o pipefail
export MICLIP_QUIET=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "attention or 336" > gpurun_out/t_attn.log 2>&1; rc=$?; tail -1 gpurun_out/t_attn.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in build/ab/libmiclip_HEAD.so aihab-clip_amd/miclip/libmiclip.so; do
  out=$(MICLIP_LIB=$L timeout -k 10 120 python scripts/bench_ops.py --ops attention --batch 128 --tokens 577 --iters 20 2>/dev/null | tail -1) || { echo fail; exit 1; }
  echo "r$r $(basename $L) $out"; done; done
bash scripts/ab_bench.sh build/ab/libmiclip_HEAD.so 2 --model ViT-L/14@336px --steps 4 --warmup 2 || exit 1
