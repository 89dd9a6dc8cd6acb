# One-head attention with the 577th key on VALU: attention tests, then op-level A/B at the
# C4 shape (HEAD library vs working tree; variants 1 and 12), 3 interleaved rounds
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/attn577ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/attn577ab/t.log 2>&1; rc=$?; tail -1 gpurun_out/attn577ab/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in build/diag/libmiclip_head.so aihab-clip_amd/miclip/libmiclip.so; do
  MICLIP_LIB=$L timeout -k 10 200 python scripts/bench_ops.py --ops attention --batch 256 --tokens 577 --width 1024 --attn-variants 1,1,12 | tail -2 | sed "s#^#$(basename $L) #" >> gpurun_out/attn577ab/ops.txt || exit 1
done; done
cat gpurun_out/attn577ab/ops.txt
