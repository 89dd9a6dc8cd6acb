# C5 (ViT-H-14 MX-fp8 bs=512) whole-step A/B: HEAD library vs working tree, 3 interleaved
# rounds, after the MX / LayerNorm tests and the C5 parity test
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/c5ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py tests/test_gpu_mx_persistent.py -x -q --timeout 120 --timeout-method thread -k "layernorm or mx" > gpurun_out/c5ab/t.log 2>&1; rc=$?; tail -1 gpurun_out/c5ab/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_openclip.py -x -q --timeout 120 --timeout-method thread -k "vith or ViT-H or openclip" > gpurun_out/c5ab/tp.log 2>&1; rc=$?; tail -1 gpurun_out/c5ab/tp.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in build/diag/libmiclip_head.so aihab-clip_amd/miclip/libmiclip.so; do
  out=$(MICLIP_LIB=$L timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --no-profile 2>/dev/null | tail -1) || { echo "bench failed ($L)"; exit 1; }
  echo "$(basename $L) $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], "clock", d.get("clock_ghz"))')" | tee -a gpurun_out/c5ab/ab.txt
done; done
