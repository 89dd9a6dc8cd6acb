set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/im2col
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k im2col > gpurun_out/im2col/t.log 2>&1; rc=$?; tail -2 gpurun_out/im2col/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/bench_ops.py --ops im2col --patch 32 > gpurun_out/im2col/ops_p32.jsonl || exit 1
timeout -k 10 120 python scripts/bench_ops.py --ops im2col --patch 14 > gpurun_out/im2col/ops_p14.jsonl || exit 1
cat gpurun_out/im2col/ops_p32.jsonl gpurun_out/im2col/ops_p14.jsonl
for r in 1 2 3; do for L in build/diag/libmiclip_head.so aihab-clip_amd/miclip/libmiclip.so; do
  out=$(MICLIP_LIB=$L timeout -k 10 200 python bench.py --model ViT-B/32 --dtype bf16 --steps 20 --warmup 3 --no-cpu-baseline --no-profile 2>/dev/null | tail -1) || { echo "bench failed ($L)"; exit 1; }
  echo "$L $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], "clock", d.get("clock_ghz"))')" | tee -a gpurun_out/im2col/c2_ab.txt
done; done
