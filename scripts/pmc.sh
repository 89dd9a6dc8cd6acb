#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, kernel-trace only, no
# other tracing) over the GEMM micro-benchmark. Output: gpurun_out/pmc/<pass>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
CMD=(python3 scripts/bench_ops.py --ops gemm --only fc,proj --variants 256,257 --iters 5)
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc/p$i" -o run -- "${CMD[@]}" > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"; tail -3 gpurun_out/pmc/p$i.log
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
done
